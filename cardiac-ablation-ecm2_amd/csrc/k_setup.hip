// k_setup.hip -- quadrature-data setup and coefficient projection (gfx950).
//
// Setup (S1..S3): qdata from element corner coordinates or from MFEM-layout Jacobians
// (PADiffusionSetup3D bilininteg_diffusion_kernels.cpp:243-367, mass setup
// bilininteg_mass_pa.cpp:60-78, GeometricFactors mesh.cpp:15220-15273); grid-function
// coefficients at the quadrature points (GridFunctionCoefficient -> CoefficientVector::Project,
// coefficient.cpp:2052-2070, qfunction.cpp:73-98) composed with the bioheat temperature laws.
#include "dev_common.hpp"

#include <type_traits>

namespace ecm2
{
namespace
{
using namespace dev;

// c(e,q) = law(T(x_q)),  T(x_q) = (B x B x B) T_e  (generic (D, Q) fallback).
__global__ void k_coeff_gridfunc(int ne, int D, int Q, const int *__restrict__ gmap, const Basis1D b,
                                 const double *__restrict__ T, int kind, double scale, double slope,
                                 double t_ref, CoeffParams cp, double *__restrict__ out)
{
   const int NQ = Q * Q * Q, ND = D * D * D;
   const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
   if (t >= (long)ne * NQ) { return; }
   const int e = (int)(t / NQ), q = (int)(t % NQ);
   const int qx = q % Q, qy = (q / Q) % Q, qz = q / (Q * Q);
   double v = 0.0;
   for (int dz = 0; dz < D; dz++)
      for (int dy = 0; dy < D; dy++)
         for (int dx = 0; dx < D; dx++)
         {
            const int g = gmap[(size_t)e * ND + (dz * D + dy) * D + dx];
            const double tv = g >= 0 ? T[g] : -T[-1 - g];
            v += b.B[qx + MQ * dx] * b.B[qy + MQ * dy] * b.B[qz + MQ * dz] * tv;
         }
   out[t] = coeff_law(kind, v, scale, slope, t_ref, cp.p);
}

// The same, sum-factorised: one wave per element, lanes (dy,dz) gather a T x-line and contract
// in x, lanes (qx,dz) in y, lanes (qx,qy) in z; out[e][q] (q = qx + Q(qy + Q qz)).
template <int D, int Q>
__global__ void __launch_bounds__(64)
k_coeff_line(int ne, const int *__restrict__ gmap, const Basis1D *__restrict__ btab, const double *__restrict__ T,
             int kind, double scale, double slope, double t_ref, CoeffParams cp, double *__restrict__ out)
{
   constexpr int ND = D * D * D, NQ = Q * Q * Q, DD = D * D, QQ = Q * Q, DQ = D * Q;
   __shared__ double s1[DD * Q];
   __shared__ double s2[D * QQ];
   const int e = blockIdx.x, t = threadIdx.x;
   if (e >= ne) { return; }
   if (t < DD)
   {
      CBasis *bp = stage_basis(btab);
      double tl[D];
#pragma unroll
      for (int dx = 0; dx < D; dx++)
      {
         const int g = gmap[(size_t)e * ND + t * D + dx];
         tl[dx] = g >= 0 ? T[g] : -T[-1 - g];
      }
#pragma unroll
      for (int qx = 0; qx < Q; qx++)
      {
         double u = 0.0;
#pragma unroll
         for (int dx = 0; dx < D; dx++) { u += bp->B[qx + MQ * dx] * tl[dx]; }
         s1[t * Q + qx] = u;
      }
   }
   __syncthreads();
   if (t < DQ)
   {
      CBasis *bp = stage_basis(btab);
      const int qx = t % Q, dz = t / Q;
      double l[D];
#pragma unroll
      for (int dy = 0; dy < D; dy++) { l[dy] = s1[(dz * D + dy) * Q + qx]; }
#pragma unroll
      for (int qy = 0; qy < Q; qy++)
      {
         double u = 0.0;
#pragma unroll
         for (int dy = 0; dy < D; dy++) { u += bp->B[qy + MQ * dy] * l[dy]; }
         s2[(dz * Q + qy) * Q + qx] = u;
      }
   }
   __syncthreads();
   if (t < QQ)
   {
      CBasis *bp = stage_basis(btab);
      double l[D];
#pragma unroll
      for (int dz = 0; dz < D; dz++) { l[dz] = s2[dz * QQ + t]; }
#pragma unroll
      for (int qz = 0; qz < Q; qz++)
      {
         double v = 0.0;
#pragma unroll
         for (int dz = 0; dz < D; dz++) { v += bp->B[qz + MQ * dz] * l[dz]; }
         out[(size_t)e * NQ + qz * QQ + t] = coeff_law(kind, v, scale, slope, t_ref, cp.p);
      }
   }
}

struct SetupCoef
{
   int has;          // integrator present
   int is_const;
   int dim;          // values per point: 1 scalar, 3 vector, 6 symmetric matrix, 9 general matrix
   double value;
   double cv[9];     // constant vector / matrix values
   const double *quad;   // [ne][nq] or [ne][nq][dim]
   const double *emask;  // element weights (1 / 0) of an attribute-marked integrator, or null
};

// coefficient of caller element e at point eq = e nq + q; an attribute marker zeroes the
// integrator on the elements it excludes (the effect of AddMultWithMarkers,
// bilinearform_ext.cpp:753-774,807-847, folded into the quadrature data)
__device__ __forceinline__ double coef_at(const SetupCoef &c, size_t eq, int e)
{
   const double v = c.is_const ? c.value : c.quad[eq];
   return c.emask ? v * c.emask[e] : v;
}
// entry i of a vector / matrix coefficient at point eq
__device__ __forceinline__ double coef_at_i(const SetupCoef &c, size_t eq, int e, int i)
{
   const double v = c.is_const ? c.cv[i] : c.quad[eq * c.dim + i];
   return c.emask ? v * c.emask[e] : v;
}

// PADiffusionSetup3D at one point (bilininteg_diffusion_kernels.cpp:270-362): D = W adj(J) M adj(J)^T
// / det J for the coefficient's coeffDim (scalar / vector: C1..C3 on the diagonal, :338-347; matrix
// 6 / 9: R = M adj(J)^T then adj(J) R, :297-336).  Returns the entries written to D: 6 symmetric
// (11,12,13,22,23,33) or, for a general matrix, 9 (D_ij at 3 i + j).
__device__ __forceinline__ int diff_point(const double J[3][3], double w, const SetupCoef &cd, size_t eq, int e,
                                          double D[9])
{
   const double J11 = J[0][0], J21 = J[1][0], J31 = J[2][0];
   const double J12 = J[0][1], J22 = J[1][1], J32 = J[2][1];
   const double J13 = J[0][2], J23 = J[1][2], J33 = J[2][2];
   const double detJ = J11 * (J22 * J33 - J32 * J23) - J21 * (J12 * J33 - J32 * J13) +
                       J31 * (J12 * J23 - J22 * J13);
   const double w_detJ = w / detJ;
   const double A11 = (J22 * J33) - (J23 * J32);
   const double A12 = (J32 * J13) - (J12 * J33);
   const double A13 = (J12 * J23) - (J22 * J13);
   const double A21 = (J31 * J23) - (J21 * J33);
   const double A22 = (J11 * J33) - (J13 * J31);
   const double A23 = (J21 * J13) - (J11 * J23);
   const double A31 = (J21 * J32) - (J31 * J22);
   const double A32 = (J31 * J12) - (J11 * J32);
   const double A33 = (J11 * J22) - (J12 * J21);
   if (cd.dim == 6 || cd.dim == 9)
   {
      const bool sym = cd.dim == 6;
      const double M11 = coef_at_i(cd, eq, e, 0), M12 = coef_at_i(cd, eq, e, 1), M13 = coef_at_i(cd, eq, e, 2);
      const double M21 = sym ? M12 : coef_at_i(cd, eq, e, 3);
      const double M22 = sym ? coef_at_i(cd, eq, e, 3) : coef_at_i(cd, eq, e, 4);
      const double M23 = sym ? coef_at_i(cd, eq, e, 4) : coef_at_i(cd, eq, e, 5);
      const double M31 = sym ? M13 : coef_at_i(cd, eq, e, 6);
      const double M32 = sym ? M23 : coef_at_i(cd, eq, e, 7);
      const double M33 = sym ? coef_at_i(cd, eq, e, 5) : coef_at_i(cd, eq, e, 8);
      const double R11 = M11 * A11 + M12 * A12 + M13 * A13;
      const double R12 = M11 * A21 + M12 * A22 + M13 * A23;
      const double R13 = M11 * A31 + M12 * A32 + M13 * A33;
      const double R21 = M21 * A11 + M22 * A12 + M23 * A13;
      const double R22 = M21 * A21 + M22 * A22 + M23 * A23;
      const double R23 = M21 * A31 + M22 * A32 + M23 * A33;
      const double R31 = M31 * A11 + M32 * A12 + M33 * A13;
      const double R32 = M31 * A21 + M32 * A22 + M33 * A23;
      const double R33 = M31 * A31 + M32 * A32 + M33 * A33;
      const double D11 = w_detJ * (A11 * R11 + A12 * R21 + A13 * R31);
      const double D12 = w_detJ * (A11 * R12 + A12 * R22 + A13 * R32);
      const double D13 = w_detJ * (A11 * R13 + A12 * R23 + A13 * R33);
      const double D22 = w_detJ * (A21 * R12 + A22 * R22 + A23 * R32);
      const double D23 = w_detJ * (A21 * R13 + A22 * R23 + A23 * R33);
      const double D33 = w_detJ * (A31 * R13 + A32 * R23 + A33 * R33);
      if (sym)
      {
         D[0] = D11; D[1] = D12; D[2] = D13; D[3] = D22; D[4] = D23; D[5] = D33;
         return 6;
      }
      D[0] = D11; D[1] = D12; D[2] = D13;
      D[3] = w_detJ * (A21 * R11 + A22 * R21 + A23 * R31);
      D[4] = D22; D[5] = D23;
      D[6] = w_detJ * (A31 * R11 + A32 * R21 + A33 * R31);
      D[7] = w_detJ * (A31 * R12 + A32 * R22 + A33 * R32);
      D[8] = D33;
      return 9;
   }
   double C1, C2, C3;
   if (cd.dim == 3)
   {
      C1 = coef_at_i(cd, eq, e, 0);
      C2 = coef_at_i(cd, eq, e, 1);
      C3 = coef_at_i(cd, eq, e, 2);
   }
   else { C1 = C2 = C3 = coef_at(cd, eq, e); }
   D[0] = w_detJ * (C1 * A11 * A11 + C2 * A12 * A12 + C3 * A13 * A13);
   D[1] = w_detJ * (C1 * A11 * A21 + C2 * A12 * A22 + C3 * A13 * A23);
   D[2] = w_detJ * (C1 * A11 * A31 + C2 * A12 * A32 + C3 * A13 * A33);
   D[3] = w_detJ * (C1 * A21 * A21 + C2 * A22 * A22 + C3 * A23 * A23);
   D[4] = w_detJ * (C1 * A21 * A31 + C2 * A22 * A32 + C3 * A23 * A33);
   D[5] = w_detJ * (C1 * A31 * A31 + C2 * A32 * A32 + C3 * A33 * A33);
   return 6;
}

__device__ __forceinline__ double det3(const double J[3][3])
{
   return J[0][0] * (J[1][1] * J[2][2] - J[2][1] * J[1][2]) - J[1][0] * (J[0][1] * J[2][2] - J[2][1] * J[0][2]) +
          J[2][0] * (J[0][1] * J[1][2] - J[1][1] * J[0][2]);
}

// Write D (6 symmetric entries, or 9 in NATIVE9) and the mass value at one quadrature point (any layout).
__device__ __forceinline__ void write_qdata(const int *pos, int kind, int nq, int e, int q, double w,
                                            const double J[3][3], const SetupCoef &cm,
                                            const SetupCoef &cd, double *qd_diff,
                                            double *qd_mass)
{
   const size_t eq = (size_t)e * nq + q;
   if (cd.has)
   {
      double D[9];
      const int n = diff_point(J, w, cd, eq, e, D);
#pragma unroll
      for (int c = 0; c < 9; c++)
      {
         if (c < n) { qd_diff[qidx_diff(pos, kind, nq, e, c, q)] = D[c]; }
      }
   }
   if (cm.has)
   {
      qd_mass[qidx_mass(pos, kind, nq, e, q)] = w * coef_at(cm, eq, e) * det3(J);
   }
}

// qdata from trilinear corners, templated on Q.  BLOCKED: threads run over (blk, q, lane)
// with the lane fastest, so for each quadrature point a wave writes 64 consecutive
// elements' entries (1 KiB per diffusion pair), the layout the apply kernel streams;
// perm maps the internal position to the caller element (geometry and coefficients are
// in caller order).  NATIVE: threads run over (e, q), q fastest.
template <int Q, bool BLOCKED>
__global__ void __launch_bounds__(256)
k_setup_nodes_t(const int *__restrict__ perm, int ne, const double *__restrict__ enodes,
                const double *__restrict__ W, const Basis1D b1, SetupCoef cm, SetupCoef cd,
                double *__restrict__ qd_diff, double *__restrict__ qd_mass, int kind)
{
   constexpr int NQ = Q * Q * Q;
   const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
   int e, q, lane = 0;
   long blk = 0;
   if (BLOCKED)
   {
      lane = (int)(t & 63);
      const long rest = t >> 6;
      q = (int)(rest % NQ);
      blk = rest / NQ;
      const int ipos = (int)(blk * 64 + lane);
      if (ipos >= ne) { return; }
      e = perm ? perm[ipos] : ipos;
   }
   else
   {
      if (t >= (long)ne * NQ) { return; }
      e = (int)(t / NQ);
      q = (int)(t % NQ);
   }
   const int qx = q % Q, qy = (q / Q) % Q, qz = q / (Q * Q);
   const double *X = enodes + (size_t)e * 24;
   double J[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
#pragma unroll
   for (int a = 0; a < 8; a++)
   {
      const int ax = a & 1, ay = (a >> 1) & 1, az = a >> 2;
      const double bx = b1.B[qx + MQ * ax], by = b1.B[qy + MQ * ay], bz = b1.B[qz + MQ * az];
      const double gx = b1.G[qx + MQ * ax], gy = b1.G[qy + MQ * ay], gz = b1.G[qz + MQ * az];
      const double dN0 = gx * by * bz, dN1 = bx * gy * bz, dN2 = bx * by * gz;
#pragma unroll
      for (int i = 0; i < 3; i++)
      {
         const double xi = X[i * 8 + a];
         J[i][0] += xi * dN0;
         J[i][1] += xi * dN1;
         J[i][2] += xi * dN2;
      }
   }
   if (!BLOCKED)
   {
      write_qdata(nullptr, kind, NQ, e, q, W[q], J, cm, cd, qd_diff, qd_mass);  // NATIVE / NATIVE9
      return;
   }
   // write_qdata's arithmetic (PADiffusionSetup3D / mass setup), blocked stores
   const size_t eq = (size_t)e * NQ + q;
   const double w = W[q];
   if (cd.has)
   {
      double D[9];
      (void)diff_point(J, w, cd, eq, e, D);  // (BLOCKED: symmetric coefficients only)
      v2d *dst = reinterpret_cast<v2d *>(qd_diff + ((size_t)blk * NQ + q) * 3 * 128) + lane;
      dst[0] = v2d{D[0], D[1]};
      dst[64] = v2d{D[2], D[3]};
      dst[128] = v2d{D[4], D[5]};
   }
   if (cm.has)
   {
      qd_mass[((size_t)blk * ((NQ + 1) / 2) + (q >> 1)) * 128 + lane * 2 + (q & 1)] = w * coef_at(cm, eq, e) * det3(J);
   }
}

// Affinity of MFEM-layout Jacobians: flag[0] = 1 when some point's J differs from its
// element's first point's by more than 1e-13 of that J's largest entry.
__global__ void k_jac_affine_check(int ne, int NQ, const double *__restrict__ Jg, int *__restrict__ flag)
{
   const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
   if (t >= (long)ne * NQ) { return; }
   const int e = (int)(t / NQ), q = (int)(t % NQ);
   double mx = 0.0, dv = 0.0;
   for (int c = 0; c < 9; c++)
   {
      const double j0 = Jg[((size_t)e * 9 + c) * NQ], jq = Jg[((size_t)e * 9 + c) * NQ + q];
      mx = fmax(mx, fabs(j0));
      dv = fmax(dv, fabs(jq - j0));
   }
   if (!(dv <= 1e-13 * mx)) { flag[0] = 1; }
}

__global__ void k_setup_jac(const int *__restrict__ pos, int kind, int ne, int NQ, const double *__restrict__ Jg,
                            const double *__restrict__ W, SetupCoef cm, SetupCoef cd,
                            double *__restrict__ qd_diff, double *__restrict__ qd_mass)
{
   const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
   if (t >= (long)ne * NQ) { return; }
   const int e = (int)(t / NQ), q = (int)(t % NQ);
   double J[3][3];
   for (int j = 0; j < 3; j++)
      for (int i = 0; i < 3; i++) { J[i][j] = Jg[(((size_t)e * 3 + j) * 3 + i) * NQ + q]; }
   write_qdata(pos, kind, NQ, e, q, W[q], J, cm, cd, qd_diff, qd_mass);
}

// Any nonzero off-diagonal C entry (C12, C13, C23: p0.y, p1.x, p2.x of the blocked [blk][3][64] pairs)?
__global__ void k_affine_offdiag(long n, int ne, const double *__restrict__ qd_fac, int *__restrict__ flag)
{
   const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
   if (t >= n || t >= ne) { return; }  // (t = blk 64 + lane: the element's position)
   const v2d *p = reinterpret_cast<const v2d *>(qd_fac + (t >> 6) * 3 * 128) + (t & 63);
   if (p[0].y != 0.0 || p[64].x != 0.0 || p[128].x != 0.0) { atomicOr(flag, 1); }
}

// AFFINE_E: C per element [e][6] = (C11, C12, C13, C22, C23, C33)
__global__ void k_affine_e_offdiag(int ne, const double *__restrict__ qd_fac, int *__restrict__ flag)
{
   const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
   if (e >= ne) { return; }
   const double *c = qd_fac + e * 6;
   if (c[1] != 0.0 || c[2] != 0.0 || c[4] != 0.0) { atomicOr(flag, 1); }
}

// AFFINE layout from the corners of parallelepiped elements (kernels.hpp).  J is the
// reference-cube edge matrix [x_100 - x_000 | x_010 - x_000 | x_001 - x_000] (the trilinear
// Jacobian of GeometricFactors, mesh.cpp:15220-15273, when the element is affine); the
// products are PADiffusionSetup3D's (bilininteg_diffusion_kernels.cpp:349-362) and the mass
// setup's (bilininteg_mass_pa.cpp:76) with the per-point factors W_q beta_q / W_q alpha_q kept
// apart from the element's C = adj(J) adj(J)^T / det J.  Threads over (blk, q, lane), lane
// fastest: each wave stores 1 KiB of pairs per point; the q = 0 threads store C.
// Jg (optional): MFEM-layout Jacobians J(q,i,j,e) instead of corners; the element's J is
// its first point's (all points agree for an affine element: checked by k_jac_affine_check).
template <int Q, bool BLOCKED>
__global__ void __launch_bounds__(256)
k_setup_affine(const int *__restrict__ perm, int ne, const double *__restrict__ enodes,
               const double *__restrict__ Jg,
               const double *__restrict__ W, SetupCoef cm, SetupCoef cd, int pw, int tsnap, int tmass,
               double *__restrict__ qd_fac, double *__restrict__ qd_pair)
{
   constexpr int NQ = Q * Q * Q;
   const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
   int lane, q, e;
   long blk;
   if (BLOCKED)
   {
      lane = (int)(t & 63);
      const long rest = t >> 6;
      q = (int)(rest % NQ);
      blk = rest / NQ;
      const int ipos = (int)(blk * 64 + lane);
      if (ipos >= ne) { return; }
      e = perm ? perm[ipos] : ipos;
   }
   else
   {
      // AFFINE_E: threads over (e, q), q fastest
      if (t >= (long)ne * NQ) { return; }
      e = (int)(t / NQ);
      q = (int)(t % NQ);
      lane = 0;
      blk = 0;
   }
   double J[3][3];
   if (Jg)
   {
#pragma unroll
      for (int j = 0; j < 3; j++)
#pragma unroll
         for (int i = 0; i < 3; i++) { J[i][j] = Jg[(((size_t)e * 3 + j) * 3 + i) * NQ]; }
   }
   else
   {
      const double *X = enodes + (size_t)e * 24;
#pragma unroll
      for (int i = 0; i < 3; i++)
      {
         J[i][0] = X[i * 8 + 1] - X[i * 8];
         J[i][1] = X[i * 8 + 2] - X[i * 8];
         J[i][2] = X[i * 8 + 4] - X[i * 8];
      }
   }
   const double J11 = J[0][0], J21 = J[1][0], J31 = J[2][0];
   const double J12 = J[0][1], J22 = J[1][1], J32 = J[2][1];
   const double J13 = J[0][2], J23 = J[1][2], J33 = J[2][2];
   const double detJ = J11 * (J22 * J33 - J32 * J23) - J21 * (J12 * J33 - J32 * J13) +
                       J31 * (J12 * J23 - J22 * J13);
   const size_t eq = (size_t)e * NQ + q;
   const double w = W[q];
   v2d pr;
   // (coefficient snapshot: the diffusion factor comes from the kernel's T' interpolation and the
   // single point value is the mass factor, none without a MassIntegrator)
   pr.x = tsnap ? (pw == 1 ? w * coef_at(cm, eq, e) * detJ : 0.0) : w * coef_at(cd, eq, e);
   pr.y = (!tsnap && pw == 2) ? w * coef_at(cm, eq, e) * detJ : 0.0;
   if (BLOCKED)
   {
      if (pw == 1) { qd_pair[((size_t)blk * NQ + q) * 64 + lane] = pr.x; }  // one value per point
      else if (pw == 2) { reinterpret_cast<v2d *>(qd_pair + ((size_t)blk * NQ + q) * 128)[lane] = pr; }
   }
   else if (pw == 1) { qd_pair[(size_t)e * NQ + q] = pr.x; }
   else if (pw == 2) { reinterpret_cast<v2d *>(qd_pair)[(size_t)e * NQ + q] = pr; }
   if (q == 0)
   {
      // (snapshot with the mass value per element, QLayout::tmass 2: the constant coefficient, or 1
      // when the kernel evaluates the mass law, times det J and the marker weight)
      if (BLOCKED && tsnap && tmass == 2 && cm.has) { qd_pair[(size_t)blk * 64 + lane] = coef_at(cm, eq, e) * detJ; }
      const double A11 = (J22 * J33) - (J23 * J32);
      const double A12 = (J32 * J13) - (J12 * J33);
      const double A13 = (J12 * J23) - (J22 * J13);
      const double A21 = (J31 * J23) - (J21 * J33);
      const double A22 = (J11 * J33) - (J13 * J31);
      const double A23 = (J21 * J13) - (J11 * J23);
      const double A31 = (J21 * J32) - (J31 * J22);
      const double A32 = (J31 * J12) - (J11 * J32);
      const double A33 = (J11 * J22) - (J12 * J21);
      const double r = 1.0 / detJ;
      v2d p0, p1, p2;
      p0.x = r * (A11 * A11 + A12 * A12 + A13 * A13);
      p0.y = r * (A11 * A21 + A12 * A22 + A13 * A23);
      p1.x = r * (A11 * A31 + A12 * A32 + A13 * A33);
      p1.y = r * (A21 * A21 + A22 * A22 + A23 * A23);
      p2.x = r * (A21 * A31 + A22 * A32 + A23 * A33);
      p2.y = r * (A31 * A31 + A32 * A32 + A33 * A33);
      if (BLOCKED)
      {
         v2d *dst = reinterpret_cast<v2d *>(qd_fac + (size_t)blk * 3 * 128) + lane;
         dst[0] = p0;
         dst[64] = p1;
         dst[128] = p2;
      }
      else
      {
         double *dst = qd_fac + (size_t)e * 6;  // (11, 12, 13, 22, 23, 33)
         dst[0] = p0.x; dst[1] = p0.y; dst[2] = p1.x; dst[3] = p1.y; dst[4] = p2.x; dst[5] = p2.y;
      }
   }
}

// TRILINEAR layout (kernels.hpp): per point the pair (W_q beta_q / det J_q, W_q alpha_q det J_q)
// -- the scalar factors of PADiffusionSetup3D's D = W beta adj(J) adj(J)^T / det J
// (bilininteg_diffusion_kernels.cpp:349-362) and of the mass setup's W alpha det J
// (bilininteg_mass_pa.cpp:76); the apply kernel evaluates adj(J) -- and, from the q = 0 threads,
// the element's trilinear-map coefficients c1..c7 of each coordinate from its lexicographic
// corners X_a (a = ax + 2 ay + 4 az): c1 = X1 - X0, c2 = X2 - X0, c3 = X4 - X0,
// c4 = X3 - X2 - X1 + X0, c5 = X5 - X4 - X1 + X0, c6 = X6 - X4 - X2 + X0,
// c7 = X7 - X6 - X5 - X3 + X4 + X2 + X1 - X0.
// BLOCKED = false: TRILINEAR_E (p >= 3 line / brick kernels), threads over (e, q), the
// coefficients [e][21] and the point values [e][q][pw].
template <int Q, bool BLOCKED>
__global__ void __launch_bounds__(256)
k_setup_trilinear(const int *__restrict__ perm, int ne, const double *__restrict__ enodes,
                  const double *__restrict__ cfit, const double *__restrict__ W, const QPts qp, SetupCoef cm,
                  SetupCoef cd, int pw, double *__restrict__ qd_geo, double *__restrict__ qd_pair)
{
   constexpr int NQ = Q * Q * Q;
   const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
   int lane = 0, q, e;
   long blk = 0;
   if (BLOCKED)
   {
      lane = (int)(t & 63);
      const long rest = t >> 6;
      q = (int)(rest % NQ);
      blk = rest / NQ;
      const int ipos = (int)(blk * 64 + lane);
      if (ipos >= ne) { return; }
      e = perm ? perm[ipos] : ipos;
   }
   else
   {
      if (t >= (long)ne * NQ) { return; }
      e = (int)(t / NQ);
      q = (int)(t % NQ);
   }
   double c[2 * kTrilinPairs];
   if (cfit)  // fitted from MFEM-layout Jacobians (k_jac_trilinear_fit)
   {
#pragma unroll
      for (int k = 0; k < 21; k++) { c[k] = cfit[(size_t)e * 21 + k]; }
   }
#pragma unroll
   for (int i = 0; i < (cfit ? 0 : 3); i++)
   {
      const double *x = enodes + (size_t)e * 24 + i * 8;
      c[0 * 3 + i] = x[1] - x[0];
      c[1 * 3 + i] = x[2] - x[0];
      c[2 * 3 + i] = x[4] - x[0];
      c[3 * 3 + i] = (x[3] - x[2]) - (x[1] - x[0]);
      c[4 * 3 + i] = (x[5] - x[4]) - (x[1] - x[0]);
      c[5 * 3 + i] = (x[6] - x[4]) - (x[2] - x[0]);
      c[6 * 3 + i] = ((x[7] - x[6]) - (x[5] - x[4])) - ((x[3] - x[2]) - (x[1] - x[0]));
   }
   c[21] = 0.0;
   // det J at the point from the map (the apply kernel's J: J[.][0] = c1 + c4 eta + c5 zeta +
   // c7 eta zeta, J[.][1] = c2 + c4 xi + c6 zeta + c7 xi zeta, J[.][2] = c3 + c5 xi + c6 eta + c7 xi eta)
   const double xi = qp.x[q % Q], et = qp.x[(q / Q) % Q], zt = qp.x[q / (Q * Q)];
   double J[3][3];
#pragma unroll
   for (int i = 0; i < 3; i++)
   {
      J[i][0] = (c[0 * 3 + i] + c[4 * 3 + i] * zt) + (c[3 * 3 + i] + c[6 * 3 + i] * zt) * et;
      J[i][1] = (c[1 * 3 + i] + c[5 * 3 + i] * zt) + (c[3 * 3 + i] + c[6 * 3 + i] * zt) * xi;
      J[i][2] = (c[2 * 3 + i] + c[5 * 3 + i] * et) + (c[4 * 3 + i] + c[6 * 3 + i] * et) * xi;
   }
   const double det = J[0][0] * (J[1][1] * J[2][2] - J[1][2] * J[2][1]) -
                      J[0][1] * (J[1][0] * J[2][2] - J[1][2] * J[2][0]) +
                      J[0][2] * (J[1][0] * J[2][1] - J[1][1] * J[2][0]);
   const size_t eq = (size_t)e * NQ + q;
   const double w = W[q];
   v2d pr;
   pr.x = w * coef_at(cd, eq, e) / det;
   pr.y = pw == 2 ? w * coef_at(cm, eq, e) * det : 0.0;
   if (!BLOCKED)
   {
      if (pw == 1) { qd_pair[eq] = pr.x; }
      else { reinterpret_cast<v2d *>(qd_pair)[eq] = pr; }
      if (q != 0) { return; }
#pragma unroll
      for (int k = 0; k < 21; k++) { qd_geo[(size_t)e * 21 + k] = c[k]; }
      return;
   }
   if (pw == 1) { qd_pair[((size_t)blk * NQ + q) * 64 + lane] = pr.x; }  // diffusion-only form
   else { reinterpret_cast<v2d *>(qd_pair + ((size_t)blk * NQ + q) * 128)[lane] = pr; }
   if (q != 0) { return; }
   v2d *dst = reinterpret_cast<v2d *>(qd_geo + (size_t)blk * kTrilinPairs * 128) + lane;
#pragma unroll
   for (int k = 0; k < kTrilinPairs; k++) { dst[k * 64] = v2d{c[2 * k], c[2 * k + 1]}; }
}

// The trilinear-map coefficients c1..c7 of every element recovered from MFEM-layout Jacobians
// J(q,i,j,e) (what the reference-side binding passes, GeometricFactors::JACOBIANS): J[i][0] =
// c1 + c4 eta + c5 zeta + c7 eta zeta is bilinear in (eta, zeta) -- four values at the rule's
// extreme points a = x_0, b = x_{Q-1} give it -- and J[i][1] / J[i][2] give c2, c6 and c3 the same
// way.  Then every point's J is compared with the fitted map's (1e-13 of the element's largest
// entry): bad[0] = 1 when some element is not a trilinear map of the reference cube (e.g. a
// curved, high-order mesh), which keeps the per-point layout.
template <int Q>
__global__ void k_jac_trilinear_fit(int ne, const double *__restrict__ Jg, const QPts qp, double *__restrict__ cfit)
{
   constexpr int NQ = Q * Q * Q;
   const int e = blockIdx.x * blockDim.x + threadIdx.x;
   if (e >= ne) { return; }
   const double a = qp.x[0], b = qp.x[Q - 1], h = b - a;
   auto J = [&](int i, int j, int qx, int qy, int qz) {
      return Jg[(((size_t)e * 3 + j) * 3 + i) * NQ + (qz * Q + qy) * Q + qx];
   };
   const int L = Q - 1;
   double *c = cfit + (size_t)e * 21;  // c[3 (k - 1) + i] = c_k of coordinate i
#pragma unroll
   for (int i = 0; i < 3; i++)
   {
      // J[i][0](eta, zeta) at (a, a), (b, a), (a, b), (b, b): c1, c4, c5, c7
      const double f00 = J(i, 0, 0, 0, 0), f10 = J(i, 0, 0, L, 0), f01 = J(i, 0, 0, 0, L), f11 = J(i, 0, 0, L, L);
      const double c7 = (f11 - f10 - f01 + f00) / (h * h);
      const double c4 = (f10 - f00) / h - c7 * a, c5 = (f01 - f00) / h - c7 * a;
      const double c1 = f00 - (c4 + c5) * a - c7 * a * a;
      // J[i][1](xi, zeta) = c2 + c4 xi + c6 zeta + c7 xi zeta: c2, c6 from (a, a), (a, b)
      const double g00 = J(i, 1, 0, 0, 0), g01 = J(i, 1, 0, 0, L);
      const double c6 = (g01 - g00) / h - c7 * a;
      const double c2 = g00 - c4 * a - c6 * a - c7 * a * a;
      // J[i][2](xi, eta) = c3 + c5 xi + c6 eta + c7 xi eta: c3 from (a, a)
      const double c3 = J(i, 2, 0, 0, 0) - c5 * a - c6 * a - c7 * a * a;
      c[0 * 3 + i] = c1; c[1 * 3 + i] = c2; c[2 * 3 + i] = c3; c[3 * 3 + i] = c4;
      c[4 * 3 + i] = c5; c[5 * 3 + i] = c6; c[6 * 3 + i] = c7;
   }
}

template <int Q>
__global__ void k_jac_trilinear_check(int ne, const double *__restrict__ Jg, const QPts qp,
                                      const double *__restrict__ cfit, int *__restrict__ bad)
{
   constexpr int NQ = Q * Q * Q;
   const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
   if (t >= (long)ne * NQ) { return; }
   const int e = (int)(t / NQ), q = (int)(t % NQ);
   const double xi = qp.x[q % Q], et = qp.x[(q / Q) % Q], zt = qp.x[q / (Q * Q)];
   const double *c = cfit + (size_t)e * 21;
   double mx = 0.0, dv = 0.0;
   for (int i = 0; i < 3; i++)
   {
      auto cf = [&](int k) { return c[3 * k + i]; };
      const double f[3] = {cf(0) + cf(3) * et + cf(4) * zt + cf(6) * et * zt,
                           cf(1) + cf(3) * xi + cf(5) * zt + cf(6) * xi * zt,
                           cf(2) + cf(4) * xi + cf(5) * et + cf(6) * xi * et};
      for (int j = 0; j < 3; j++)
      {
         const double v = Jg[(((size_t)e * 3 + j) * 3 + i) * NQ + q];
         mx = fmax(mx, fabs(v));
         dv = fmax(dv, fabs(v - f[j]));
      }
   }
   if (!(dv <= 1e-13 * mx)) { bad[0] = 1; }
}

// TRILINEAR -> BLOCKED: the full per-point qdata of a TRILINEAR form (for the diagonal, the
// E-vector apply and the qdata export; the apply kernel evaluates the same algebra on the fly).
// BLOCKED = false: TRILINEAR_E -> NATIVE ([e][6][NQ], [e][NQ]).
template <int Q, bool BLOCKED>
__global__ void __launch_bounds__(256)
k_trilinear_expand(int ne, const double *__restrict__ qd_geo, const double *__restrict__ qd_pair, const QPts qp,
                   int pw, double *__restrict__ qd_diff, double *__restrict__ qd_mass)
{
   constexpr int NQ = Q * Q * Q;
   const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
   int lane = 0, q, e = 0;
   long blk = 0;
   double c[2 * kTrilinPairs];
   if (BLOCKED)
   {
      lane = (int)(t & 63);
      const long rest = t >> 6;
      q = (int)(rest % NQ);
      blk = rest / NQ;
      if (blk * 64 + lane >= ne) { return; }
      const double *cg = qd_geo + (size_t)blk * kTrilinPairs * 128 + lane * 2;
#pragma unroll
      for (int k = 0; k < kTrilinPairs; k++) { c[2 * k] = cg[k * 128]; c[2 * k + 1] = cg[k * 128 + 1]; }
   }
   else
   {
      if (t >= (long)ne * NQ) { return; }
      e = (int)(t / NQ);
      q = (int)(t % NQ);
#pragma unroll
      for (int k = 0; k < 21; k++) { c[k] = qd_geo[(size_t)e * 21 + k]; }
   }
   auto cf = [&](int k, int i) { return c[3 * k + i]; };
   const double xi = qp.x[q % Q], et = qp.x[(q / Q) % Q], zt = qp.x[q / (Q * Q)];
   double J[3][3];
#pragma unroll
   for (int i = 0; i < 3; i++)
   {
      J[i][0] = (cf(0, i) + cf(4, i) * zt) + (cf(3, i) + cf(6, i) * zt) * et;
      J[i][1] = (cf(1, i) + cf(5, i) * zt) + (cf(3, i) + cf(6, i) * zt) * xi;
      J[i][2] = (cf(2, i) + cf(5, i) * et) + (cf(4, i) + cf(6, i) * et) * xi;
   }
   const double A11 = J[1][1] * J[2][2] - J[1][2] * J[2][1], A12 = J[2][1] * J[0][2] - J[0][1] * J[2][2],
                A13 = J[0][1] * J[1][2] - J[1][1] * J[0][2];
   const double A21 = J[2][0] * J[1][2] - J[1][0] * J[2][2], A22 = J[0][0] * J[2][2] - J[0][2] * J[2][0],
                A23 = J[1][0] * J[0][2] - J[0][0] * J[1][2];
   const double A31 = J[1][0] * J[2][1] - J[2][0] * J[1][1], A32 = J[2][0] * J[0][1] - J[0][0] * J[2][1],
                A33 = J[0][0] * J[1][1] - J[0][1] * J[1][0];
   v2d pr;
   if (BLOCKED)
   {
      pr = pw == 2 ? reinterpret_cast<const v2d *>(qd_pair + ((size_t)blk * NQ + q) * 128)[lane]
                   : v2d{qd_pair[((size_t)blk * NQ + q) * 64 + lane], 0.0};
   }
   else
   {
      const size_t eq = (size_t)e * NQ + q;
      pr = pw == 2 ? reinterpret_cast<const v2d *>(qd_pair)[eq] : v2d{qd_pair[eq], 0.0};
   }
   const double sc = pr.x;  // W beta / det J
   v2d p0, p1, p2;
   p0.x = sc * (A11 * A11 + A12 * A12 + A13 * A13);
   p0.y = sc * (A11 * A21 + A12 * A22 + A13 * A23);
   p1.x = sc * (A11 * A31 + A12 * A32 + A13 * A33);
   p1.y = sc * (A21 * A21 + A22 * A22 + A23 * A23);
   p2.x = sc * (A21 * A31 + A22 * A32 + A23 * A33);
   p2.y = sc * (A31 * A31 + A32 * A32 + A33 * A33);
   if (!BLOCKED)
   {
      double *d = qd_diff + (size_t)e * 6 * NQ + q;  // (11, 12, 13, 22, 23, 33)
      d[0] = p0.x; d[NQ] = p0.y; d[2 * NQ] = p1.x; d[3 * NQ] = p1.y; d[4 * NQ] = p2.x; d[5 * NQ] = p2.y;
      if (pw == 2) { qd_mass[(size_t)e * NQ + q] = pr.y; }
      return;
   }
   v2d *dst = reinterpret_cast<v2d *>(qd_diff + ((size_t)blk * NQ + q) * 3 * 128) + lane;
   dst[0] = p0;
   dst[64] = p1;
   dst[128] = p2;
   if (pw == 2) { qd_mass[((size_t)blk * ((NQ + 1) / 2) + (q >> 1)) * 128 + lane * 2 + (q & 1)] = pr.y; }  // W alpha det J
}

// AFFINE (p <= 2) -> BLOCKED: D(q) = (W beta)_q C_e and the mass value (W alpha det J)_q, for the
// diagonal, the E-vector apply and the qdata export of a diffusion-only AFFINE form (pw = 1).
// BLOCKED = false: AFFINE_E -> NATIVE ([e][6][NQ], [e][NQ]).
template <int Q, bool BLOCKED>
__global__ void __launch_bounds__(256)
k_affine_expand(int ne, const double *__restrict__ qd_fac, const double *__restrict__ qd_pair, int pw,
                double *__restrict__ qd_diff, double *__restrict__ qd_mass, const double *__restrict__ qm1)
{
   // qm1 (BLOCKED, optional): the mass values one per point ([blk][q][lane], a coefficient-snapshot
   // form's stored W alpha det J) for qd_mass
   constexpr int NQ = Q * Q * Q;
   const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
   if (!BLOCKED)
   {
      if (t >= (long)ne * NQ) { return; }
      const int e = (int)(t / NQ), q = (int)(t % NQ);
      const size_t eq = (size_t)e * NQ + q;
      const v2d pr = pw == 2 ? reinterpret_cast<const v2d *>(qd_pair)[eq] : v2d{qd_pair[eq], 0.0};
#pragma unroll
      for (int k = 0; k < 6; k++) { qd_diff[((size_t)e * 6 + k) * NQ + q] = pr.x * qd_fac[(size_t)e * 6 + k]; }
      if (pw == 2) { qd_mass[eq] = pr.y; }
      return;
   }
   const int lane = (int)(t & 63);
   const long rest = t >> 6;
   const int q = (int)(rest % NQ);
   const long blk = rest / NQ;
   if (blk * 64 + lane >= ne) { return; }
   const v2d *C = reinterpret_cast<const v2d *>(qd_fac + (size_t)blk * 3 * 128) + lane;
   const v2d pr = pw == 2 ? reinterpret_cast<const v2d *>(qd_pair + ((size_t)blk * NQ + q) * 128)[lane]
                          : v2d{qd_pair[((size_t)blk * NQ + q) * 64 + lane], 0.0};
   v2d *dst = reinterpret_cast<v2d *>(qd_diff + ((size_t)blk * NQ + q) * 3 * 128) + lane;
#pragma unroll
   for (int k = 0; k < 3; k++) { dst[k * 64] = pr.x * C[k * 64]; }
   if (pw == 2 || qm1)
   {
      qd_mass[((size_t)blk * ((NQ + 1) / 2) + (q >> 1)) * 128 + lane * 2 + (q & 1)] =
         qm1 ? qm1[((size_t)blk * NQ + q) * 64 + lane] : pr.y;
   }
}

// The coefficient snapshot T' = A + B T of an affine law of an H1 field (k_apply_tpe_ts).
__global__ void __launch_bounds__(256) k_affine_snapshot(int n, const double *__restrict__ T, double A, double B,
                                                         double *__restrict__ out)
{
   const int i = blockIdx.x * blockDim.x + threadIdx.x;
   if (i < n) { out[i] = A + B * T[i]; }
}

// The same snapshot in block lattice-slot order, out[b][j] = A + B T[lmap[b][j]] (lattice-map blocks:
// the snapshot kernel then reads it contiguously instead of a second dependent gather), and back to
// dof order (every dof is some block's lattice point; shared points carry equal values).
__global__ void __launch_bounds__(256) k_affine_snapshot_lattice(long n, int nlp, const int *__restrict__ lmap,
                                                                 const double *__restrict__ T, double A, double B,
                                                                 double *__restrict__ out)
{
   const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
   if (i < n) { out[i] = A + B * T[lmap[i] & 0x3fffffff]; }
}

__global__ void __launch_bounds__(256) k_lattice_to_dofs(long n, const int *__restrict__ lmap,
                                                         const double *__restrict__ v, double *__restrict__ out)
{
   const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
   if (i < n) { out[lmap[i] & 0x3fffffff] = v[i]; }
}

// AFFINE with a coefficient snapshot -> BLOCKED (the diagonal, the E-vector apply, the qdata export):
// D(q) = W_q beta_q C_e with beta_q the snapshot's law at the point (caller order [e][q]) and the stored
// element matrices C_e; the mass W alpha det J as stored per point (tmass 1) or W_q (alpha_q | 1) times
// the stored per-element (c alpha) det J (tmass 2; alpha_q null: a constant, folded in).
template <int Q>
__global__ void __launch_bounds__(256)
k_tsnap_expand(const int *__restrict__ perm, int ne, const double *__restrict__ W, const double *__restrict__ qd_fac,
               const double *__restrict__ qd_m, int tmass, const double *__restrict__ beta_q,
               const double *__restrict__ alpha_q, double *__restrict__ qd_diff, double *__restrict__ qd_mass)
{
   constexpr int NQ = Q * Q * Q;
   const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
   const int lane = (int)(t & 63);
   const long rest = t >> 6;
   const int q = (int)(rest % NQ);
   const long blk = rest / NQ;
   const int ipos = (int)(blk * 64 + lane);
   if (ipos >= ne) { return; }
   const int e = perm ? perm[ipos] : ipos;
   const size_t eq = (size_t)e * NQ + q;
   const double wb = W[q] * beta_q[eq];
   const v2d *C = reinterpret_cast<const v2d *>(qd_fac + (size_t)blk * 3 * 128) + lane;
   v2d *dst = reinterpret_cast<v2d *>(qd_diff + ((size_t)blk * NQ + q) * 3 * 128) + lane;
#pragma unroll
   for (int k = 0; k < 3; k++) { dst[k * 64] = wb * C[k * 64]; }
   if (tmass == 0) { return; }
   const double m = tmass == 1 ? qd_m[((size_t)blk * NQ + q) * 64 + lane]
                               : W[q] * (alpha_q ? alpha_q[eq] : 1.0) * qd_m[(size_t)blk * 64 + lane];
   qd_mass[((size_t)blk * ((NQ + 1) / 2) + (q >> 1)) * 128 + lane * 2 + (q & 1)] = m;
}

// Element weights applied to one integrator's stored qdata, any layout (the marker diagonal,
// PAForm::assemble_diagonal): every entry of integrator `integ` on caller element e is multiplied
// by w[e].  pos: caller element -> internal position (blocked layouts), else null.
__global__ void __launch_bounds__(256)
k_scale_elements(int kind, int ne, int NQ, int pw, int tsnap, int tmass, const int *__restrict__ pos, int integ,
                 const double *__restrict__ w, double *__restrict__ qdd, double *__restrict__ qdm)
{
   const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
   if (t >= (long)ne * NQ) { return; }
   const int e = (int)(t / NQ), q = (int)(t % NQ);
   const double wt = w[e];
   if (wt == 1.0) { return; }
   const int ip = pos ? pos[e] : e;
   const size_t blk = (size_t)(ip >> 6);
   const int lane = ip & 63;
   const size_t eq = (size_t)e * NQ + q, bq = (blk * NQ + q) * 64 + lane;
   const bool diff = integ == 1;
   switch (kind)
   {
   case QLAYOUT_NATIVE:
   case QLAYOUT_NATIVE9:
      if (diff)
      {
         const int nc = kind == QLAYOUT_NATIVE9 ? 9 : 6;
         for (int c = 0; c < nc; c++) { qdd[((size_t)e * nc + c) * NQ + q] *= wt; }
      }
      else { qdm[eq] *= wt; }
      break;
   case QLAYOUT_BLOCKED:
      if (diff)
      {
         for (int k = 0; k < 3; k++)
         {
            double *p = qdd + ((blk * NQ + q) * 3 + k) * 128 + lane * 2;
            p[0] *= wt;
            p[1] *= wt;
         }
      }
      else { qdm[(blk * ((NQ + 1) / 2) + (q >> 1)) * 128 + lane * 2 + (q & 1)] *= wt; }
      break;
   case QLAYOUT_AFFINE:
      if (diff)
      {
         if (q != 0) { break; }
         for (int k = 0; k < 3; k++)  // the element matrix C_e
         {
            double *p = qdd + (blk * 3 + k) * 128 + lane * 2;
            p[0] *= wt;
            p[1] *= wt;
         }
      }
      else if (pw == 2) { qdm[bq * 2 + 1] *= wt; }
      else if (tsnap && tmass == 2) { if (q == 0) { qdm[blk * 64 + lane] *= wt; } }  // per element
      else if (tsnap && pw == 1) { qdm[bq] *= wt; }  // W alpha det J alone (coefficient snapshot)
      break;
   case QLAYOUT_AFFINE_E:
      if (diff)
      {
         if (q == 0) { for (int k = 0; k < 6; k++) { qdd[(size_t)e * 6 + k] *= wt; } }
      }
      else if (pw == 2) { qdm[eq * 2 + 1] *= wt; }
      break;
   case QLAYOUT_TRILINEAR:
      if (diff) { qdm[pw == 2 ? bq * 2 : bq] *= wt; }  // W beta / det J
      else if (pw == 2) { qdm[bq * 2 + 1] *= wt; }
      break;
   case QLAYOUT_TRILINEAR_E:
      if (diff) { qdm[pw == 2 ? eq * 2 : eq] *= wt; }
      else if (pw == 2) { qdm[eq * 2 + 1] *= wt; }
      break;
   default: break;
   }
}

SetupCoef make_setup_coef(const CoeffDesc *c, const double *q)
{
   SetupCoef s{};
   if (!c) { return s; }
   s.has = 1;
   s.is_const = (c->kind == COEFF_CONSTANT || (c->kind >= COEFF_CONST_VECTOR && c->kind <= COEFF_CONST_MATRIX));
   s.dim = c->dim();
   s.value = c->value;
   for (int i = 0; i < 9; i++) { s.cv[i] = c->cv[i]; }
   s.quad = q;
   s.emask = c->emask;
   return s;
}

} // namespace

namespace kern
{

void coeff_gridfunc(int ne, int D, int Q, const int *gmap, const Basis1D &b, const Basis1D *btab, const CoeffDesc &c,
                    double *out, hipStream_t s)
{
   const long n = (long)ne * Q * Q * Q;
   if (n == 0) { return; }
   CoeffParams cp;
   for (int i = 0; i < 6; i++) { cp.p[i] = c.p[i]; }
#define ECM2_COEFF_CASE(DD, QQ)                                                                         \
   if (D == DD && Q == QQ)                                                                              \
   {                                                                                                    \
      hipLaunchKernelGGL((k_coeff_line<DD, QQ>), dim3(ne), dim3(64), 0, s, ne, gmap, btab, c.lvec, c.kind, \
                         c.scale, c.slope, c.t_ref, cp, out);                                          \
      ECM2_HIP(hipGetLastError());                                                                      \
      return;                                                                                           \
   }
   if (btab)
   {
      ECM2_COEFF_CASE(2, 3) ECM2_COEFF_CASE(3, 4) ECM2_COEFF_CASE(4, 5) ECM2_COEFF_CASE(5, 6)
      ECM2_COEFF_CASE(6, 7) ECM2_COEFF_CASE(7, 8) ECM2_COEFF_CASE(2, 2) ECM2_COEFF_CASE(3, 3)
      ECM2_COEFF_CASE(4, 4) ECM2_COEFF_CASE(5, 5)
   }
#undef ECM2_COEFF_CASE
   hipLaunchKernelGGL(k_coeff_gridfunc, dim3(grid_for(n, 256)), dim3(256), 0, s, ne, D, Q, gmap, b, c.lvec, c.kind,
                      c.scale, c.slope, c.t_ref, cp, out);
   ECM2_HIP(hipGetLastError());
}

void setup_from_nodes(const QLayout &L, int Q, const double *enodes, const double *W,
                      const Basis1D &b1, const CoeffDesc *cm, const CoeffDesc *cd,
                      const double *cm_q, const double *cd_q, double *qd_diff,
                      double *qd_mass, hipStream_t s)
{
   const long n = (long)L.ne * L.nq;
   if (n == 0) { return; }
   const SetupCoef scm = make_setup_coef(cm, cm_q), scd = make_setup_coef(cd, cd_q);
   const bool blocked = L.kind == QLAYOUT_BLOCKED;
   ECM2_VERIFY(!blocked || !L.pos || L.perm, ERR_INTERNAL, "blocked setup needs the inverse permutation");
   const long nb = blocked ? (long)L.nblk() * 64 * L.nq : n;
#define ECM2_SETUP_CASE(QQ)                                                                              \
   if (Q == QQ)                                                                                          \
   {                                                                                                     \
      if (blocked)                                                                                       \
      {                                                                                                  \
         hipLaunchKernelGGL((k_setup_nodes_t<QQ, true>), dim3(grid_for(nb, 256)), dim3(256), 0, s, L.perm, L.ne, \
                            enodes, W, b1, scm, scd, qd_diff, qd_mass, L.kind);                          \
      }                                                                                                  \
      else                                                                                               \
      {                                                                                                  \
         hipLaunchKernelGGL((k_setup_nodes_t<QQ, false>), dim3(grid_for(nb, 256)), dim3(256), 0, s, nullptr, L.ne, \
                            enodes, W, b1, scm, scd, qd_diff, qd_mass, L.kind);                          \
      }                                                                                                  \
      ECM2_HIP(hipGetLastError());                                                                       \
      return;                                                                                            \
   }
   ECM2_SETUP_CASE(2) ECM2_SETUP_CASE(3) ECM2_SETUP_CASE(4) ECM2_SETUP_CASE(5)
   ECM2_SETUP_CASE(6) ECM2_SETUP_CASE(7) ECM2_SETUP_CASE(8)
#undef ECM2_SETUP_CASE
   ECM2_VERIFY(false, ERR_UNSUPPORTED, "setup: Q1D " << Q << " not instantiated");
}

void tsnap_expand(const QLayout &L, int Q, const double *W, const double *qd_fac, const double *qd_m,
                  const double *beta_q, const double *alpha_q, double *qd_diff, double *qd_mass, hipStream_t s)
{
   ECM2_VERIFY(L.kind == QLAYOUT_AFFINE && L.tsnap && Q == 4, ERR_INTERNAL, "snapshot expansion: AFFINE p = 2");
   const long n = (long)L.nblk() * 64 * L.nq;
   if (n == 0) { return; }
   hipLaunchKernelGGL((k_tsnap_expand<4>), dim3(grid_for(n, 256)), dim3(256), 0, s, L.perm, L.ne, W, qd_fac, qd_m,
                      L.tmass, beta_q, alpha_q, qd_diff, qd_mass);
   ECM2_HIP(hipGetLastError());
}

void scale_elements(const QLayout &L, int integ, const double *w, double *qd_diff, double *qd_mass, hipStream_t s)
{
   const long n = (long)L.ne * L.nq;
   if (n == 0) { return; }
   hipLaunchKernelGGL(k_scale_elements, dim3(grid_for(n, 256)), dim3(256), 0, s, L.kind, L.ne, L.nq, L.pw, L.tsnap, L.tmass,
                      L.blocked() ? L.pos : nullptr, integ, w, qd_diff, qd_mass);
   ECM2_HIP(hipGetLastError());
}

void affine_snapshot(int n, const double *T, double A, double B, double *out, hipStream_t s)
{
   if (n == 0) { return; }
   hipLaunchKernelGGL(k_affine_snapshot, dim3(grid_for(n, 256)), dim3(256), 0, s, n, T, A, B, out);
   ECM2_HIP(hipGetLastError());
}

void affine_snapshot_lattice(int nblk, int nlp, const int *lmap, const double *T, double A, double B, double *out,
                             hipStream_t s)
{
   const long n = (long)nblk * nlp;
   if (n == 0) { return; }
   hipLaunchKernelGGL(k_affine_snapshot_lattice, dim3(grid_for(n, 256)), dim3(256), 0, s, n, nlp, lmap, T, A, B, out);
   ECM2_HIP(hipGetLastError());
}

void lattice_to_dofs(int nblk, int nlp, const int *lmap, const double *v, double *out, hipStream_t s)
{
   const long n = (long)nblk * nlp;
   if (n == 0) { return; }
   hipLaunchKernelGGL(k_lattice_to_dofs, dim3(grid_for(n, 256)), dim3(256), 0, s, n, lmap, v, out);
   ECM2_HIP(hipGetLastError());
}

bool jacobians_affine(int ne, int nq, const double *J, hipStream_t s)
{
   if (ne == 0) { return true; }
   DeviceArray<int> flag;
   flag.resize(1);
   ECM2_HIP(hipMemsetAsync(flag.data(), 0, sizeof(int), s));
   const long n = (long)ne * nq;
   hipLaunchKernelGGL(k_jac_affine_check, dim3(grid_for(n, 256)), dim3(256), 0, s, ne, nq, J, flag.data());
   ECM2_HIP(hipGetLastError());
   int h = 1;
   ECM2_HIP(hipMemcpyAsync(&h, flag.data(), sizeof(int), hipMemcpyDeviceToHost, s));
   ECM2_HIP(hipStreamSynchronize(s));
   return h == 0;
}

bool jacobians_trilinear_fit(int ne, int Q, const QPts &qp, const double *J, double *cfit, hipStream_t s)
{
   if (ne == 0) { return true; }
   DeviceArray<int> flag;
   flag.resize(1);
   ECM2_HIP(hipMemsetAsync(flag.data(), 0, sizeof(int), s));
   const long n = (long)ne * Q * Q * Q;
   bool done = false;
#define ECM2_FIT(QQ)                                                                                           \
   if (Q == QQ)                                                                                                \
   {                                                                                                           \
      hipLaunchKernelGGL((k_jac_trilinear_fit<QQ>), dim3(grid_for(ne, 256)), dim3(256), 0, s, ne, J, qp, cfit);   \
      hipLaunchKernelGGL((k_jac_trilinear_check<QQ>), dim3(grid_for(n, 256)), dim3(256), 0, s, ne, J, qp, cfit,   \
                         flag.data());                                                                        \
      done = true;                                                                                             \
   }
   ECM2_FIT(2) ECM2_FIT(3) ECM2_FIT(4) ECM2_FIT(5) ECM2_FIT(6) ECM2_FIT(7) ECM2_FIT(8)
#undef ECM2_FIT
   if (!done) { return false; }
   ECM2_HIP(hipGetLastError());
   int h = 1;
   ECM2_HIP(hipMemcpyAsync(&h, flag.data(), sizeof(int), hipMemcpyDeviceToHost, s));
   ECM2_HIP(hipStreamSynchronize(s));
   return h == 0;
}

// the launches of a (Q, BLOCKED) kernel family over n threads; BLOCKED: the p <= 2 layouts
#define ECM2_Q_BLOCKED_CASES(KERNEL, n, blocked, ...)                                                      \
   {                                                                                                       \
      bool done_ = false;                                                                                  \
      auto launch_ = [&](auto qc) {                                                                        \
         constexpr int QQ = decltype(qc)::value;                                                           \
         if (blocked)                                                                                      \
         {                                                                                                 \
            hipLaunchKernelGGL((KERNEL<QQ, true>), dim3(grid_for(n, 256)), dim3(256), 0, s, __VA_ARGS__);  \
         }                                                                                                 \
         else { hipLaunchKernelGGL((KERNEL<QQ, false>), dim3(grid_for(n, 256)), dim3(256), 0, s, __VA_ARGS__); } \
         done_ = true;                                                                                     \
      };                                                                                                   \
      switch (Q)                                                                                           \
      {                                                                                                    \
      case 2: launch_(std::integral_constant<int, 2>()); break;                                            \
      case 3: launch_(std::integral_constant<int, 3>()); break;                                            \
      case 4: launch_(std::integral_constant<int, 4>()); break;                                            \
      case 5: launch_(std::integral_constant<int, 5>()); break;                                            \
      case 6: launch_(std::integral_constant<int, 6>()); break;                                            \
      case 7: launch_(std::integral_constant<int, 7>()); break;                                            \
      case 8: launch_(std::integral_constant<int, 8>()); break;                                            \
      default: break;                                                                                      \
      }                                                                                                    \
      ECM2_VERIFY(done_, ERR_UNSUPPORTED, #KERNEL ": Q1D " << Q << " not instantiated");                  \
      ECM2_HIP(hipGetLastError());                                                                         \
   }

void setup_trilinear(const QLayout &L, int Q, const double *enodes, const double *cfit, const double *W,
                     const QPts &qp, const CoeffDesc *cm, const CoeffDesc *cd, const double *cm_q, const double *cd_q,
                     double *qd_geo, double *qd_pair, hipStream_t s)
{
   if (L.ne == 0) { return; }
   ECM2_VERIFY((L.kind == QLAYOUT_TRILINEAR || L.kind == QLAYOUT_TRILINEAR_E) && (cm || L.pw == 1) && cd &&
                  (enodes || cfit),
               ERR_INTERNAL, "trilinear setup needs a TRILINEAR layout, the coefficients and the corners or fitted maps");
   ECM2_VERIFY(!L.pos || L.perm, ERR_INTERNAL, "blocked setup needs the inverse permutation");
   const SetupCoef scm = make_setup_coef(cm, cm_q), scd = make_setup_coef(cd, cd_q);
   const bool blk = L.kind == QLAYOUT_TRILINEAR;
   const long n = blk ? (long)L.nblk() * 64 * L.nq : (long)L.ne * L.nq;
   const int *perm = blk ? L.perm : nullptr;
   ECM2_Q_BLOCKED_CASES(k_setup_trilinear, n, blk, perm, L.ne, enodes, cfit, W, qp, scm, scd, L.pw, qd_geo, qd_pair)
}

void trilinear_expand(const QLayout &L, int Q, const double *qd_geo, const double *qd_pair, const QPts &qp,
                      double *qd_diff, double *qd_mass, hipStream_t s)
{
   if (L.ne == 0) { return; }
   const bool blk = L.kind == QLAYOUT_TRILINEAR;
   const long n = blk ? (long)L.nblk() * 64 * L.nq : (long)L.ne * L.nq;
   ECM2_Q_BLOCKED_CASES(k_trilinear_expand, n, blk, L.ne, qd_geo, qd_pair, qp, L.pw, qd_diff, qd_mass)
}

void affine_expand(const QLayout &L, int Q, const double *qd_fac, const double *qd_pair, double *qd_diff,
                   double *qd_mass, hipStream_t s, const double *qm1)
{
   ECM2_VERIFY(!qm1 || L.kind == QLAYOUT_AFFINE, ERR_INTERNAL, "single mass values: blocked layout");
   if (L.ne == 0) { return; }
   const bool blk = L.kind == QLAYOUT_AFFINE;
   const long n = blk ? (long)L.nblk() * 64 * L.nq : (long)L.ne * L.nq;
   ECM2_Q_BLOCKED_CASES(k_affine_expand, n, blk, L.ne, qd_fac, qd_pair, L.pw, qd_diff, qd_mass, qm1)
}
#undef ECM2_Q_BLOCKED_CASES

bool affine_c_diagonal(const QLayout &L, const double *qd_fac, int *dflag, hipStream_t s)
{
   ECM2_VERIFY(L.kind == QLAYOUT_AFFINE || L.kind == QLAYOUT_AFFINE_E, ERR_INTERNAL,
               "C diagonal test: AFFINE / AFFINE_E layouts only");
   if (L.ne == 0) { return true; }
   ECM2_HIP(hipMemsetAsync(dflag, 0, sizeof(int), s));
   if (L.kind == QLAYOUT_AFFINE)
   {
      const long n = (long)L.nblk() * 64;
      hipLaunchKernelGGL(k_affine_offdiag, dim3(grid_for(n, 256)), dim3(256), 0, s, n, L.ne, qd_fac, dflag);
   }
   else { hipLaunchKernelGGL(k_affine_e_offdiag, dim3(grid_for(L.ne, 256)), dim3(256), 0, s, L.ne, qd_fac, dflag); }
   ECM2_HIP(hipGetLastError());
   int h = 1;
   ECM2_HIP(hipMemcpyAsync(&h, dflag, sizeof(int), hipMemcpyDeviceToHost, s));
   ECM2_HIP(hipStreamSynchronize(s));
   return h == 0;
}

void setup_affine(const QLayout &L, int Q, const double *enodes, const double *J, const double *W,
                  const CoeffDesc *cm, const CoeffDesc *cd, const double *cm_q, const double *cd_q,
                  double *qd_fac, double *qd_pair, hipStream_t s)
{
   if (L.ne == 0) { return; }
   ECM2_VERIFY(L.affine() && cd && (cm || L.pw <= 1) && (!L.tsnap || L.kind == QLAYOUT_AFFINE), ERR_INTERNAL,
               "affine setup needs an AFFINE layout and its coefficients");
   ECM2_VERIFY(!L.pos || L.perm, ERR_INTERNAL, "blocked setup needs the inverse permutation");
   const SetupCoef scm = make_setup_coef(cm, cm_q), scd = make_setup_coef(cd, cd_q);
   const bool blk = L.kind == QLAYOUT_AFFINE;
   const long n = blk ? (long)L.nblk() * 64 * L.nq : (long)L.ne * L.nq;
#define ECM2_AFF_CASE(QQ)                                                                               \
   if (Q == QQ)                                                                                          \
   {                                                                                                     \
      if (blk)                                                                                           \
      {                                                                                                  \
         hipLaunchKernelGGL((k_setup_affine<QQ, true>), dim3(grid_for(n, 256)), dim3(256), 0, s, L.perm, L.ne, \
                            enodes, J, W, scm, scd, L.pw, L.tsnap, L.tmass, qd_fac, qd_pair);            \
      }                                                                                                  \
      else                                                                                               \
      {                                                                                                  \
         hipLaunchKernelGGL((k_setup_affine<QQ, false>), dim3(grid_for(n, 256)), dim3(256), 0, s, nullptr, L.ne, \
                            enodes, J, W, scm, scd, L.pw, L.tsnap, L.tmass, qd_fac, qd_pair);                     \
      }                                                                                                  \
      ECM2_HIP(hipGetLastError());                                                                       \
      return;                                                                                            \
   }
   ECM2_AFF_CASE(2) ECM2_AFF_CASE(3) ECM2_AFF_CASE(4) ECM2_AFF_CASE(5) ECM2_AFF_CASE(6) ECM2_AFF_CASE(7)
   ECM2_AFF_CASE(8)
#undef ECM2_AFF_CASE
   ECM2_VERIFY(false, ERR_UNSUPPORTED, "affine setup: Q1D " << Q << " not instantiated");
}

void setup_from_jacobians(const QLayout &L, const double *J, const double *W,
                          const CoeffDesc *cm, const CoeffDesc *cd, const double *cm_q,
                          const double *cd_q, double *qd_diff, double *qd_mass, hipStream_t s)
{
   const long n = (long)L.ne * L.nq;
   if (n == 0) { return; }
   hipLaunchKernelGGL(k_setup_jac, dim3(grid_for(n, 256)), dim3(256), 0, s, L.pos, L.kind, L.ne, L.nq,
                      J, W, make_setup_coef(cm, cm_q), make_setup_coef(cd, cd_q), qd_diff,
                      qd_mass);
   ECM2_HIP(hipGetLastError());
}

} // namespace kern
} // namespace ecm2
