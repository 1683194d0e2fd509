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
   std::vector<double> qw1;    // 1D Gauss-Legendre weights (W = qw1[qx] qw1[qy] qw1[qz])
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

// Even/odd split of the 1D tables (round 3, the brick kernel's contractions).  The GLL nodes and
// the Gauss points are symmetric about the element midpoint, so B(Q-1-q, D-1-d) = B(q, d) and
// G(Q-1-q, D-1-d) = -G(q, d).  For a table T and i < D/2:
//   TP(q, i) = (T(q, i) + T(q, D-1-i)) / 2,  TM(q, i) = (T(q, i) - T(q, D-1-i)) / 2,
// and TP(q, D/2) = T(q, D/2) for odd D.  A contraction y = T x of a line then needs the rows
// q < Q/2 only, on e_i = x_i + x_{D-1-i} and o_i = x_i - x_{D-1-i}:
//   B: y_q, y_{Q-1-q} = (BP e) +- (BM o)      G: y_q, y_{Q-1-q} = (GM o) +- (GP e)
// (and the transposes likewise): about (D+1)/2 + D/2 instead of D multiply-adds per pair of
// outputs (the even-odd decomposition of sum-factorised tensor kernels).  The identity is exact
// algebra for the table rows it uses; the mirrored rows are the symmetric images, equal to the
// computed ones up to rounding (~1e-16 relative).
struct BasisEO
{
   double BP[MAX_Q1D * MAX_D1D], BM[MAX_Q1D * MAX_D1D];  // [q + MAX_Q1D * i]
   double GP[MAX_Q1D * MAX_D1D], GM[MAX_Q1D * MAX_D1D];
};
// The device copy of the tables the line / brick / diagonal / coefficient kernels read (as a
// Basis1D through the first member; the brick kernel also reads eo).
struct BasisDev
{
   Basis1D b;
   BasisEO eo;
};
BasisDev make_basis_dev(const Basis1D &b, int D, int Q);

} // namespace ecm2
