// fe.hpp -- 1D quadrature rules and the H1 Gauss-Lobatto tensor basis tables.
//
// Host-side setup (reference row a8): the B/G tables every PA kernel consumes.
//   Gauss-Legendre points/weights     fem/intrules.cpp:424-495
//   Gauss-Lobatto points/weights      fem/intrules.cpp:497-640
//   barycentric Lagrange basis        fem/fe/fe_base.cpp:1733-1768, 1858-1936
//   tensor DofToQuad B[q+Q*d], G      fem/fe/fe_base.cpp:2619-2662
//   default rule size Q1D = p + 2      bilininteg.cpp:1347-1366, 1450-1462, intrules.cpp:1181-1200
#pragma once

#include <vector>

namespace ecm2
{

constexpr int MAX_D1D = 8;
constexpr int MAX_Q1D = 8;

void gauss_legendre(int np, double *x, double *w);
void gauss_lobatto(int np, double *x, double *w);
void basis_eval(int p, const double *nodes, double y, double *u, double *d);

// Default quadrature size for Mass+Diffusion on trilinear hexes.
int default_q1d(int order);

struct DofToQuad
{
   int ndof = 0, nqpt = 0;
   std::vector<double> B, G;   // [q + nqpt*d]
   std::vector<double> W;      // tensor weights, [qx + Q*(qy + Q*qz)]
   std::vector<double> qpts;   // 1D Gauss-Legendre points
   std::vector<double> nodes;  // 1D GLL nodes
};

DofToQuad make_dof_to_quad(int order, int q1d);

// Kernel-argument copy of the 1D tables (lands in the kernarg segment, read
// with scalar loads; fully unrolled kernels index it with constants).
struct Basis1D
{
   double B[MAX_Q1D * MAX_D1D];
   double G[MAX_Q1D * MAX_D1D];
};
Basis1D make_basis1d(const DofToQuad &m);

} // namespace ecm2
