// fe.cpp -- see fe.hpp for the reference citations.
#include "fe.hpp"
#include "common.hpp"

#include <cmath>

namespace ecm2
{

void gauss_legendre(int np, double *x, double *w)
{
   // Closed forms for 1..3 points, Newton on P_n otherwise (intrules.cpp:430-495).
   switch (np)
   {
      case 1: x[0] = 0.5; w[0] = 1.0; return;
      case 2:
         x[0] = 0.21132486540518711775; w[0] = 0.5;
         x[1] = 0.78867513459481288225; w[1] = 0.5;
         return;
      case 3:
         x[0] = 0.11270166537925831148; w[0] = 5. / 18.;
         x[1] = 0.5;                    w[1] = 4. / 9.;
         x[2] = 0.88729833462074168852; w[2] = 5. / 18.;
         return;
      default: break;
   }
   const int n = np, half = (n + 1) / 2;
   for (int i = 1; i <= half; i++)
   {
      double z = std::cos(M_PI * (i - 0.25) / (n + 0.5));
      double pp = 0, p1 = 0, p2 = 0, xi = 0.;
      bool converged = false;
      for (;;)
      {
         p2 = 1;
         p1 = z;
         for (int j = 2; j <= n; j++)
         {
            const double p3 = p2;
            p2 = p1;
            p1 = ((2 * j - 1) * z * p2 - (j - 1) * p3) / j;
         }
         pp = n * (z * p1 - p2) / (z * z - 1);
         if (converged) { break; }
         const double dz = p1 / pp;
         if (std::fabs(dz) < 1e-16)
         {
            converged = true;
            xi = ((1 - z) + dz) / 2;
         }
         z -= dz;
      }
      x[i - 1] = xi;
      x[n - i] = 1 - xi;
      w[i - 1] = w[n - i] = 1. / (4 * xi * (1 - xi) * pp * pp);
   }
}

void gauss_lobatto(int np, double *x, double *w)
{
   if (np == 1) { x[0] = 0.5; w[0] = 1.0; return; }
   x[0] = 0.0;
   x[np - 1] = 1.0;
   w[0] = w[np - 1] = 1.0 / (np * (np - 1));
   for (int i = 1; i <= (np - 1) / 2; ++i)
   {
      // Chebyshev initial guess, Newton on (x^2-1) P'_{np-1} (intrules.cpp:560-620)
      double xi = std::sin(M_PI * ((double)i / (np - 1) - 0.5));
      double zi = 0., pl = 0., plm1 = 0.;
      bool converged = false;
      for (int iter = 0; iter < 64; ++iter)
      {
         plm1 = 1.0;
         pl = xi;
         for (int l = 1; l < np - 1; ++l)
         {
            const double plp1 = ((2 * l + 1) * xi * pl - l * plm1) / (l + 1);
            plm1 = pl;
            pl = plp1;
         }
         if (converged) { break; }
         const double dx = (xi * pl - plm1) / (np * pl);
         if (std::fabs(dx) < 1e-16)
         {
            converged = true;
            zi = ((1.0 + xi) - dx) / 2;
         }
         xi -= dx;
      }
      ECM2_VERIFY(converged, ERR_INTERNAL, "Gauss-Lobatto Newton iteration failed, np=" << np);
      x[i] = zi;
      w[i] = 1.0 / (np * (np - 1) * pl * pl);
      x[np - 1 - i] = 1.0 - zi;
      w[np - 1 - i] = w[i];
   }
}

void basis_eval(int p, const double *x, double y, double *u, double *d)
{
   if (p == 0) { u[0] = 1.0; d[0] = 0.0; return; }
   double bw[MAX_D1D + 2];
   for (int i = 0; i <= p; i++) { bw[i] = 1.0; }
   for (int i = 0; i <= p; i++)
   {
      for (int j = 0; j < i; j++)
      {
         const double xij = x[i] - x[j];
         bw[i] *= xij;
         bw[j] *= -xij;
      }
   }
   for (int i = 0; i <= p; i++) { bw[i] = 1.0 / bw[i]; }
   // Locate the node interval containing y; lk = prod_{i != k}(y - x_i).
   int k;
   double lk = 1.0;
   for (k = 0; k < p; k++)
   {
      if (y >= (x[k] + x[k + 1]) / 2) { lk *= y - x[k]; }
      else
      {
         for (int i = k + 1; i <= p; i++) { lk *= y - x[i]; }
         break;
      }
   }
   const double l = lk * (y - x[k]);
   double sk = 0.0;
   int i;
   for (i = 0; i < k; i++)
   {
      const double si = 1.0 / (y - x[i]);
      sk += si;
      u[i] = l * si * bw[i];
   }
   u[k] = lk * bw[k];
   for (i++; i <= p; i++)
   {
      const double si = 1.0 / (y - x[i]);
      sk += si;
      u[i] = l * si * bw[i];
   }
   const double lp = l * sk + lk;
   for (i = 0; i < k; i++) { d[i] = (lp * bw[i] - u[i]) / (y - x[i]); }
   d[k] = sk * u[k];
   for (i++; i <= p; i++) { d[i] = (lp * bw[i] - u[i]) / (y - x[i]); }
}

int default_q1d(int order)
{
   const int rule_order = (2 * order + 2) | 1;
   return rule_order / 2 + 1;
}

DofToQuad make_dof_to_quad(int order, int q1d)
{
   ECM2_VERIFY(order >= 1 && order + 1 <= MAX_D1D, ERR_ARG, "unsupported order " << order);
   ECM2_VERIFY(q1d >= 1 && q1d <= MAX_Q1D, ERR_ARG, "unsupported q1d " << q1d);
   DofToQuad m;
   m.ndof = order + 1;
   m.nqpt = q1d;
   m.nodes.resize(m.ndof);
   std::vector<double> nw(m.ndof), qw(q1d);
   m.qpts.resize(q1d);
   gauss_lobatto(m.ndof, m.nodes.data(), nw.data());
   gauss_legendre(q1d, m.qpts.data(), qw.data());
   m.B.resize(q1d * m.ndof);
   m.G.resize(q1d * m.ndof);
   double u[MAX_D1D], d[MAX_D1D];
   for (int q = 0; q < q1d; q++)
   {
      basis_eval(order, m.nodes.data(), m.qpts[q], u, d);
      for (int j = 0; j < m.ndof; j++)
      {
         m.B[q + q1d * j] = u[j];
         m.G[q + q1d * j] = d[j];
      }
   }
   m.qw1 = qw;
   m.W.resize(q1d * q1d * q1d);
   for (int iz = 0; iz < q1d; ++iz)
      for (int iy = 0; iy < q1d; ++iy)
         for (int ix = 0; ix < q1d; ++ix)
         {
            m.W[(iz * q1d + iy) * q1d + ix] = qw[ix] * qw[iy] * qw[iz];
         }
   return m;
}

Basis1D make_basis1d(const DofToQuad &m)
{
   Basis1D b{};
   // Repack with the compile-time stride MAX_Q1D so kernels index B[q + MAX_Q1D*d].
   for (int d = 0; d < m.ndof; d++)
      for (int q = 0; q < m.nqpt; q++)
      {
         b.B[q + MAX_Q1D * d] = m.B[q + m.nqpt * d];
         b.G[q + MAX_Q1D * d] = m.G[q + m.nqpt * d];
      }
   return b;
}

BasisDev make_basis_dev(const Basis1D &b, int D, int Q)
{
   BasisDev t{};
   t.b = b;
   const int H = D / 2;
   for (int q = 0; q < Q; q++)
   {
      for (int i = 0; i < H; i++)
      {
         const int a = q + MAX_Q1D * i, r = q + MAX_Q1D * (D - 1 - i);
         t.eo.BP[a] = 0.5 * (b.B[a] + b.B[r]);
         t.eo.BM[a] = 0.5 * (b.B[a] - b.B[r]);
         t.eo.GP[a] = 0.5 * (b.G[a] + b.G[r]);
         t.eo.GM[a] = 0.5 * (b.G[a] - b.G[r]);
      }
      if (D % 2)
      {
         const int a = q + MAX_Q1D * H;
         t.eo.BP[a] = b.B[a];
         t.eo.GP[a] = b.G[a];
      }
   }
   return t;
}

} // namespace ecm2
