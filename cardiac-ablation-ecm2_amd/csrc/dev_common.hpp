// dev_common.hpp -- device-side helpers shared by the gfx950 kernel translation units
// (k_setup.hip, k_tpe.hip, k_line.hip, k_misc.hip).  Included by .hip files only.
#pragma once

#include "kernels.hpp"

#include <hip/hip_runtime.h>

namespace ecm2
{
namespace dev
{

constexpr int MQ = MAX_Q1D;
typedef double v2d __attribute__((ext_vector_type(2)));
typedef double v4d __attribute__((ext_vector_type(4)));

inline unsigned grid_for(long n, int bs) { return (unsigned)((n + bs - 1) / bs); }


// pos: caller element -> internal position (element permutation of the blocked layout)
__device__ __forceinline__ size_t qidx_diff(const int *pos, int kind, int nq, int e, int c, int q)
{
   if (kind == QLAYOUT_NATIVE) { return ((size_t)e * 6 + c) * nq + q; }
   if (kind == QLAYOUT_NATIVE9) { return ((size_t)e * 9 + c) * nq + q; }
   if (pos) { e = pos[e]; }
   const int blk = e >> 6, lane = e & 63;
   return (((size_t)blk * nq + q) * 3 + (c >> 1)) * 128 + lane * 2 + (c & 1);
}

__device__ __forceinline__ size_t qidx_mass(const int *pos, int kind, int nq, int e, int q)
{
   if (kind == QLAYOUT_NATIVE || kind == QLAYOUT_NATIVE9) { return (size_t)e * nq + q; }
   if (pos) { e = pos[e]; }
   const int blk = e >> 6, lane = e & 63;
   const int nqh = (nq + 1) >> 1;
   return ((size_t)blk * nqh + (q >> 1)) * 128 + lane * 2 + (q & 1);
}

// Value of diffusion entry c / mass at (e, q) in any layout; AFFINE recombines the
// per-point scalar W beta (qdm pair .x) with the element matrix C (qdd), and stores the mass
// value as the pair's .y.
__device__ __forceinline__ size_t affine_pair(const int *pos, int nq, int e, int q)
{
   if (pos) { e = pos[e]; }
   return (((size_t)(e >> 6) * nq + q) * 64 + (e & 63)) * 2;
}
__device__ __forceinline__ double qd_diff_at(const double *qdd, const double *qdm, const int *pos, int kind,
                                             int nq, int e, int c, int q)
{
   // (NATIVE9: c = 3 i + j of the general D_ij; every other layout: the symmetric c = 0..5)
   if (kind == QLAYOUT_NATIVE9) { return qdd[((size_t)e * 9 + c) * nq + q]; }
   if (kind == QLAYOUT_AFFINE_E) { return qdm[((size_t)e * nq + q) * 2] * qdd[(size_t)e * 6 + c]; }
   if (kind == QLAYOUT_AFFINE)
   {
      const int ie = pos ? pos[e] : e;
      return qdm[affine_pair(nullptr, nq, ie, q)] * qdd[(((size_t)(ie >> 6) * 3 + (c >> 1)) * 64 + (ie & 63)) * 2 + (c & 1)];
   }
   return qdd[qidx_diff(pos, kind, nq, e, c, q)];
}
// The diffusion term k of the PA diagonal's sum over i, j of D_ij (d_i phi)(d_j phi) at (e, q):
// k = 0..5 -> D_11, D_22, D_33, D_12 + D_21, D_13 + D_31, D_23 + D_32 (PADiffusionDiagonal3D,
// bilininteg_diffusion_kernels.hpp:410-431: symmetric ? ksym : 3 i + j).
__device__ __forceinline__ double qd_diag_term(const double *qdd, const double *qdm, const int *pos, int kind,
                                               int nq, int e, int k, int q)
{
   if (kind == QLAYOUT_NATIVE9)
   {
      const int a[6] = {0, 4, 8, 1, 2, 5}, b[6] = {-1, -1, -1, 3, 6, 7};
      const double v = qd_diff_at(qdd, qdm, pos, kind, nq, e, a[k], q);
      return b[k] < 0 ? v : v + qd_diff_at(qdd, qdm, pos, kind, nq, e, b[k], q);
   }
   const int src[6] = {0, 3, 5, 1, 2, 4};  // symmetric (11,12,13,22,23,33)
   const double v = qd_diff_at(qdd, qdm, pos, kind, nq, e, src[k], q);
   return k >= 3 ? 2.0 * v : v;
}

__device__ __forceinline__ double qd_mass_at(const double *qdm, const int *pos, int kind, int nq, int e, int q)
{
   if (kind == QLAYOUT_NATIVE9) { return qdm[(size_t)e * nq + q]; }
   if (kind == QLAYOUT_AFFINE_E) { return qdm[((size_t)e * nq + q) * 2 + 1]; }
   if (kind == QLAYOUT_AFFINE) { return qdm[affine_pair(pos, nq, e, q) + 1]; }
   return qdm[qidx_mass(pos, kind, nq, e, q)];
}

__device__ __forceinline__ int dof_of(int g) { return g >= 0 ? g : -1 - g; }

// adj(J) of a 3x3 Jacobian (rows A_i = (A_i1, A_i2, A_i3)): PADiffusionSetup3D's
// adjugate (bilininteg_diffusion_kernels.cpp:349-360), so D = (W beta / det J) A A^T.
__device__ __forceinline__ void adj3(const double (&J)[3][3], double (&A)[3][3])
{
   A[0][0] = J[1][1] * J[2][2] - J[1][2] * J[2][1];
   A[0][1] = J[2][1] * J[0][2] - J[0][1] * J[2][2];
   A[0][2] = J[0][1] * J[1][2] - J[1][1] * J[0][2];
   A[1][0] = J[2][0] * J[1][2] - J[1][0] * J[2][2];
   A[1][1] = J[0][0] * J[2][2] - J[0][2] * J[2][0];
   A[1][2] = J[1][0] * J[0][2] - J[0][0] * J[1][2];
   A[2][0] = J[1][0] * J[2][1] - J[2][0] * J[1][1];
   A[2][1] = J[2][0] * J[0][1] - J[0][0] * J[2][1];
   A[2][2] = J[0][0] * J[1][1] - J[0][1] * J[1][0];
}

// The trilinear map's Jacobian at (xi, eta, zeta) from its coefficients c[3 (k - 1) + i] = c_k of
// coordinate i (kernels.hpp TRILINEAR): J[i][0] = c1 + c4 eta + c5 zeta + c7 eta zeta, J[i][1] =
// c2 + c4 xi + c6 zeta + c7 xi zeta, J[i][2] = c3 + c5 xi + c6 eta + c7 xi eta.
__device__ __forceinline__ void trilinear_jacobian(const double *c, double xi, double et, double zt,
                                                   double (&J)[3][3])
{
#pragma unroll
   for (int i = 0; i < 3; i++)
   {
      J[i][0] = (c[i] + c[12 + i] * zt) + (c[9 + i] + c[18 + i] * zt) * et;
      J[i][1] = (c[3 + i] + c[15 + i] * zt) + (c[9 + i] + c[18 + i] * zt) * xi;
      J[i][2] = (c[6 + i] + c[15 + i] * et) + (c[12 + i] + c[18 + i] * et) * xi;
   }
}

// The six symmetric entries (11, 12, 13, 22, 23, 33) of D = sc A A^T, A = adj(J).
__device__ __forceinline__ void trilinear_dmat(const double (&J)[3][3], double sc, double (&d)[6])
{
   double A[3][3];
   adj3(J, A);
   d[0] = sc * (A[0][0] * A[0][0] + A[0][1] * A[0][1] + A[0][2] * A[0][2]);
   d[1] = sc * (A[0][0] * A[1][0] + A[0][1] * A[1][1] + A[0][2] * A[1][2]);
   d[2] = sc * (A[0][0] * A[2][0] + A[0][1] * A[2][1] + A[0][2] * A[2][2]);
   d[3] = sc * (A[1][0] * A[1][0] + A[1][1] * A[1][1] + A[1][2] * A[1][2]);
   d[4] = sc * (A[1][0] * A[2][0] + A[1][1] * A[2][1] + A[1][2] * A[2][2]);
   d[5] = sc * (A[2][0] * A[2][0] + A[2][1] * A[2][1] + A[2][2] * A[2][2]);
}

// Encoded (fused-kernel) map entries: bits 0-29 dof, bit 30 "shared" (the dof is held by
// more than one entry of the whole mesh after the kernel's own face assembly -> partial slot
// or atomic add), bit 31 orientation sign.
__device__ __forceinline__ int bdof(int g) { return g & 0x3fffffff; }
__device__ __forceinline__ bool bneg(int g) { return g < 0; }
__device__ __forceinline__ bool bshared(int g) { return (g >> 30) & 1; }

// XCD-aware workgroup order: the hardware deals workgroup i to XCD i % 8 (MI355X_MICROARCH.md,
// "Workgroup dispatch"); remapping i to a contiguous range per XCD keeps neighbouring work items
// (which share x values and partial-slot lines) in one XCD's L2.  A bijection on [0, G) for any G.
__device__ __forceinline__ int xcd_contiguous(int i, int G)
{
   const int q = G >> 3, r = G & 7, x = i & 7, j = i >> 3;
   return x * q + (x < r ? x : r) + j;
}

// Basis tables for the line / brick / diagonal / coefficient kernels: a device copy of the
// (D1D, Q1D) Basis1D read through the constant address space, with the pointer laundered per
// stage (asm barrier) so the compiler issues scalar loads where the entries are used instead
// of hoisting 2 D Q doubles out of the element loop (which exceeds the SGPR file).
typedef const __attribute__((address_space(4))) Basis1D CBasis;

__device__ __forceinline__ CBasis *stage_basis(const Basis1D *tab)
{
   CBasis *p = (CBasis *)tab;
   asm volatile("" : "+s"(p));
   return p;
}

} // namespace dev
} // namespace ecm2
