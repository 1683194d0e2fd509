// pa_kernels.hip -- hand-written gfx950 (CDNA4) kernels for the PA diffusion+mass path.
//
// Hot path (reference K1..K5, SURVEY §2 "Device kernels on the path"):
//   k_apply_tpe   fused gather -> B/G contractions -> Pennes/heat-capacity and
//                 conductivity weighting -> transposed contractions -> scatter,
//                 one THREAD per element, 64 elements per wave.  Replaces
//                 ElementRestriction::Mult (restriction.cpp:109-129), the mass
//                 and diffusion AddMultPA kernels (bilininteg_mass_kernels.hpp:809-1033,
//                 bilininteg_diffusion_kernels.hpp:989-1214) and
//                 ElementRestriction::MultTranspose (restriction.cpp:152-186) in
//                 one pass over HBM.  qdata (95% of the bytes) is streamed once with
//                 1 KiB-per-wave-instruction dwordx4 loads; the 1D contractions run
//                 in registers (no LDS, no cross-lane traffic); the L-vector scatter
//                 uses hardware FP64 atomics (global_atomic_add_f64).
//   k_apply_wpe   one WORKGROUP per element (lane per quadrature point, LDS
//                 between the six 1D stages), any order; also serves the
//                 reference-shaped unfused API (E-vector in/out).
// Setup (S1..S3): qdata from element corner coordinates or from MFEM-layout
// Jacobians (PADiffusionSetup3D bilininteg_diffusion_kernels.cpp:243-367,
// mass setup bilininteg_mass_pa.cpp:60-78, GeometricFactors mesh.cpp:15220-15273).
#include "kernels.hpp"

#include <mutex>
#include <set>
#include <tuple>

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

namespace ecm2
{
namespace
{

constexpr int MQ = MAX_Q1D;
constexpr int kDefaultTpeVariant = 4;  // pipelined + brick merge
typedef double v2d __attribute__((ext_vector_type(2)));

// pos: caller element -> internal position (element permutation of the blocked layout)
__device__ __forceinline__ size_t qidx_diff(const int *pos, int kind, int nq, int e, int c, int q)
{
   if (kind == QLAYOUT_NATIVE) { return ((size_t)e * 6 + c) * nq + q; }
   if (pos) { e = pos[e]; }
   const int blk = e >> 6, lane = e & 63;
   return (((size_t)blk * nq + q) * 3 + (c >> 1)) * 128 + lane * 2 + (c & 1);
}

__device__ __forceinline__ size_t qidx_mass(const int *pos, int kind, int nq, int e, int q)
{
   if (kind == QLAYOUT_NATIVE) { return (size_t)e * nq + q; }
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
   if (kind == QLAYOUT_AFFINE_E) { return qdm[((size_t)e * nq + q) * 2] * qdd[(size_t)e * 6 + c]; }
   if (kind == QLAYOUT_AFFINE)
   {
      const int ie = pos ? pos[e] : e;
      return qdm[affine_pair(nullptr, nq, ie, q)] * qdd[(((size_t)(ie >> 6) * 3 + (c >> 1)) * 64 + (ie & 63)) * 2 + (c & 1)];
   }
   return qdd[qidx_diff(pos, kind, nq, e, c, q)];
}
__device__ __forceinline__ double qd_mass_at(const double *qdm, const int *pos, int kind, int nq, int e, int q)
{
   if (kind == QLAYOUT_AFFINE_E) { return qdm[((size_t)e * nq + q) * 2 + 1]; }
   if (kind == QLAYOUT_AFFINE) { return qdm[affine_pair(pos, nq, e, q) + 1]; }
   return qdm[qidx_mass(pos, kind, nq, e, q)];
}

__device__ __forceinline__ int dof_of(int g) { return g >= 0 ? g : -1 - g; }

// Blocked (fused-kernel) map entries: bits 0-29 dof, bit 30 "shared" (the dof is held by
// more than one lane of the whole mesh after in-wave assembly -> atomic add), bit 31 sign.
__device__ __forceinline__ int bdof(int g) { return g & 0x3fffffff; }
__device__ __forceinline__ bool bneg(int g) { return g < 0; }
__device__ __forceinline__ bool bshared(int g) { return (g >> 30) & 1; }

// --------------------------------------------------------------------------
// Setup kernels
// --------------------------------------------------------------------------

// c(e,q) = scale * (1 + slope * (T(x_q) - t_ref)),  T(x_q) = (B x B x B) T_e.
__global__ void k_coeff_gridfunc(int ne, int D, int Q, const int *__restrict__ gmap,
                                 const Basis1D b, const double *__restrict__ T, double scale,
                                 double slope, double t_ref, double *__restrict__ out)
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
   out[t] = scale * (1.0 + slope * (v - t_ref));
}

struct SetupCoef
{
   int has;          // integrator present
   int is_const;
   double value;
   const double *quad;
};

__device__ __forceinline__ double coef_at(const SetupCoef &c, size_t eq)
{
   return c.is_const ? c.value : c.quad[eq];
}

// Write D (6 symmetric entries) and mass value at one quadrature point.
__device__ __forceinline__ void write_qdata(const int *pos, int kind, int nq, int e, int q, double w,
                                            const double J[3][3], const SetupCoef &cm,
                                            const SetupCoef &cd, double *qd_diff,
                                            double *qd_mass)
{
   const double J11 = J[0][0], J21 = J[1][0], J31 = J[2][0];
   const double J12 = J[0][1], J22 = J[1][1], J32 = J[2][1];
   const double J13 = J[0][2], J23 = J[1][2], J33 = J[2][2];
   const double detJ = J11 * (J22 * J33 - J32 * J23) - J21 * (J12 * J33 - J32 * J13) +
                       J31 * (J12 * J23 - J22 * J13);
   const size_t eq = (size_t)e * nq + q;
   if (cd.has)
   {
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
      const double C = coef_at(cd, eq);
      qd_diff[qidx_diff(pos, kind, nq, e, 0, q)] = w_detJ * (C * A11 * A11 + C * A12 * A12 + C * A13 * A13);
      qd_diff[qidx_diff(pos, kind, nq, e, 1, q)] = w_detJ * (C * A11 * A21 + C * A12 * A22 + C * A13 * A23);
      qd_diff[qidx_diff(pos, kind, nq, e, 2, q)] = w_detJ * (C * A11 * A31 + C * A12 * A32 + C * A13 * A33);
      qd_diff[qidx_diff(pos, kind, nq, e, 3, q)] = w_detJ * (C * A21 * A21 + C * A22 * A22 + C * A23 * A23);
      qd_diff[qidx_diff(pos, kind, nq, e, 4, q)] = w_detJ * (C * A21 * A31 + C * A22 * A32 + C * A23 * A33);
      qd_diff[qidx_diff(pos, kind, nq, e, 5, q)] = w_detJ * (C * A31 * A31 + C * A32 * A32 + C * A33 * A33);
   }
   if (cm.has)
   {
      qd_mass[qidx_mass(pos, kind, nq, e, q)] = w * coef_at(cm, eq) * detJ;
   }
}

__global__ void k_setup_nodes(const int *__restrict__ pos, int kind, int ne, int Q, const double *__restrict__ enodes,
                              const double *__restrict__ W, const Basis1D b1, SetupCoef cm,
                              SetupCoef cd, double *__restrict__ qd_diff,
                              double *__restrict__ qd_mass)
{
   const int NQ = Q * Q * Q;
   const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
   if (t >= (long)ne * NQ) { return; }
   const int e = (int)(t / NQ), q = (int)(t % NQ);
   const int qx = q % Q, qy = (q / Q) % Q, qz = q / (Q * Q);
   const double *X = enodes + (size_t)e * 24;
   double J[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
   for (int a = 0; a < 8; a++)
   {
      const int ax = a & 1, ay = (a >> 1) & 1, az = a >> 2;
      const double bx = b1.B[qx + MQ * ax], by = b1.B[qy + MQ * ay], bz = b1.B[qz + MQ * az];
      const double gx = b1.G[qx + MQ * ax], gy = b1.G[qy + MQ * ay], gz = b1.G[qz + MQ * az];
      const double dN0 = gx * by * bz, dN1 = bx * gy * bz, dN2 = bx * by * gz;
      for (int i = 0; i < 3; i++)
      {
         const double xi = X[i * 8 + a];
         J[i][0] += xi * dN0;
         J[i][1] += xi * dN1;
         J[i][2] += xi * dN2;
      }
   }
   write_qdata(pos, kind, NQ, e, q, W[q], J, cm, cd, qd_diff, qd_mass);
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
                double *__restrict__ qd_diff, double *__restrict__ qd_mass)
{
   constexpr int NQ = Q * Q * Q;
   const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
   int e, q, ipos = 0, lane = 0;
   long blk = 0;
   if (BLOCKED)
   {
      lane = (int)(t & 63);
      const long rest = t >> 6;
      q = (int)(rest % NQ);
      blk = rest / NQ;
      ipos = (int)(blk * 64 + lane);
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
      write_qdata(nullptr, QLAYOUT_NATIVE, NQ, e, q, W[q], J, cm, cd, qd_diff, qd_mass);
      return;
   }
   // same arithmetic as write_qdata (PADiffusionSetup3D / mass setup), blocked stores
   const double J11 = J[0][0], J21 = J[1][0], J31 = J[2][0];
   const double J12 = J[0][1], J22 = J[1][1], J32 = J[2][1];
   const double J13 = J[0][2], J23 = J[1][2], J33 = J[2][2];
   const double detJ = J11 * (J22 * J33 - J32 * J23) - J21 * (J12 * J33 - J32 * J13) +
                       J31 * (J12 * J23 - J22 * J13);
   const size_t eq = (size_t)e * NQ + q;
   const double w = W[q];
   if (cd.has)
   {
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
      const double C = coef_at(cd, eq);
      v2d p0, p1, p2;
      p0.x = w_detJ * (C * A11 * A11 + C * A12 * A12 + C * A13 * A13);
      p0.y = w_detJ * (C * A11 * A21 + C * A12 * A22 + C * A13 * A23);
      p1.x = w_detJ * (C * A11 * A31 + C * A12 * A32 + C * A13 * A33);
      p1.y = w_detJ * (C * A21 * A21 + C * A22 * A22 + C * A23 * A23);
      p2.x = w_detJ * (C * A21 * A31 + C * A22 * A32 + C * A23 * A33);
      p2.y = w_detJ * (C * A31 * A31 + C * A32 * A32 + C * A33 * A33);
      v2d *dst = reinterpret_cast<v2d *>(qd_diff + ((size_t)blk * NQ + q) * 3 * 128) + lane;
      dst[0] = p0;
      dst[64] = p1;
      dst[128] = p2;
   }
   if (cm.has)
   {
      qd_mass[((size_t)blk * ((NQ + 1) / 2) + (q >> 1)) * 128 + lane * 2 + (q & 1)] = w * coef_at(cm, eq) * detJ;
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
               const double *__restrict__ W, SetupCoef cm, SetupCoef cd, double *__restrict__ qd_fac,
               double *__restrict__ qd_pair)
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
   pr.x = w * coef_at(cd, eq);
   pr.y = w * coef_at(cm, eq) * detJ;
   if (BLOCKED) { reinterpret_cast<v2d *>(qd_pair + ((size_t)blk * NQ + q) * 128)[lane] = pr; }
   else { reinterpret_cast<v2d *>(qd_pair)[(size_t)e * NQ + q] = pr; }
   if (q == 0)
   {
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

// --------------------------------------------------------------------------
// Fused apply, thread per element (blocked layout)
// --------------------------------------------------------------------------

// Per-(qy,qz) products of the 1D tables, [qz][qy][kind][dz][dy] with kind
// 0: B(qy,dy)B(qz,dz)  1: G(qy,dy)B(qz,dz)  2: B(qy,dy)G(qz,dz).  Read by uniform
// (scalar-cache) loads inside the row loop, so they cost no VGPRs.
struct RowTable
{
   const double *p;
};

template <int D, int Q, bool MASS, bool DIFF, bool SPLIT>
__global__ void __launch_bounds__(256)
k_apply_tpe(int ne, int blk_begin, int blk_end, int n_owned, const int *__restrict__ gmap,
            const double *__restrict__ qdd, const double *__restrict__ qdm,
            const double *__restrict__ x, const double *__restrict__ xg,
            double *__restrict__ y, double *__restrict__ yg, const Basis1D b,
            const double *__restrict__ rowtab)
{
   constexpr int ND = D * D * D, NQ = Q * Q * Q, NQH = (NQ + 1) / 2, DD = D * D;
   const int lane = threadIdx.x & 63;
   const int blk = blk_begin + blockIdx.x * 4 + (threadIdx.x >> 6);
   if (blk >= blk_end) { return; }  // wave-uniform
   const int e = blk * 64 + lane;
   const bool active = e < ne;
   const int *mp = gmap + (size_t)blk * ND * 64 + lane;

   // ---- gather (ElementRestriction::Mult); SPLIT: [owned | ghost] local L-vector ----
   double X[ND];
#pragma unroll
   for (int a = 0; a < ND; a++)
   {
      const int g = mp[a * 64];
      const int d = bdof(g);
      const double v = (!SPLIT || d < n_owned) ? x[d] : xg[d - n_owned];
      X[a] = bneg(g) ? -v : v;
   }
   double Yo[ND];
#pragma unroll
   for (int a = 0; a < ND; a++) { Yo[a] = 0.0; }

   const double *qd = qdd + (size_t)blk * NQ * 3 * 128 + lane * 2;
   const double *qm = qdm + (size_t)blk * NQH * 128 + lane * 2;

#pragma unroll 1
   for (int row = 0; row < Q * Q; row++)   // row = qy + Q*qz (wave-uniform)
   {
      const double *P = rowtab + (size_t)row * 3 * DD;   // uniform -> s_load
      // qdata of the row's Q points: issue all loads first
      v2d dq[Q][3];
      double mq[Q];
#pragma unroll
      for (int qx = 0; qx < Q; qx++)
      {
         const int q = row * Q + qx;
         if (DIFF)
         {
#pragma unroll
            for (int k = 0; k < 3; k++)
            {
               dq[qx][k] = __builtin_nontemporal_load(
                  reinterpret_cast<const v2d *>(qd + ((size_t)q * 3 + k) * 128));
            }
         }
         if (MASS)
         {
            mq[qx] = qm[(size_t)(q >> 1) * 128 + (q & 1)];
         }
      }
      // forward: Y00 = (B_y B_z) X, Y01 = (G_y B_z) X, Y10 = (B_y G_z) X
      double Y00[D], Y01[D], Y10[D];
#pragma unroll
      for (int dx = 0; dx < D; dx++)
      {
         double u = 0.0, v = 0.0, w = 0.0;
#pragma unroll
         for (int dz = 0; dz < D; dz++)
#pragma unroll
            for (int dy = 0; dy < D; dy++)
            {
               const double c = X[(dz * D + dy) * D + dx];
               u += P[0 * DD + dz * D + dy] * c;
               if (DIFF)
               {
                  v += P[1 * DD + dz * D + dy] * c;
                  w += P[2 * DD + dz * D + dy] * c;
               }
            }
         Y00[dx] = u; Y01[dx] = v; Y10[dx] = w;
      }
      double T0[D], T1[D], T2[D];
#pragma unroll
      for (int dx = 0; dx < D; dx++) { T0[dx] = 0.0; T1[dx] = 0.0; T2[dx] = 0.0; }
#pragma unroll
      for (int qx = 0; qx < Q; qx++)
      {
         double u = 0.0, ux = 0.0, uy = 0.0, uz = 0.0;
#pragma unroll
         for (int dx = 0; dx < D; dx++)
         {
            const double bq = b.B[qx + MQ * dx], gq = b.G[qx + MQ * dx];
            if (MASS) { u += bq * Y00[dx]; }
            if (DIFF)
            {
               ux += gq * Y00[dx];
               uy += bq * Y01[dx];
               uz += bq * Y10[dx];
            }
         }
         double m = 0.0, fx = 0.0, fy = 0.0, fz = 0.0;
         if (MASS) { m = mq[qx] * u; }
         if (DIFF)
         {
            // (11,12) (13,22) (23,33)
            const v2d d0 = dq[qx][0], d1 = dq[qx][1], d2 = dq[qx][2];
            fx = d0.x * ux + d0.y * uy + d1.x * uz;
            fy = d0.y * ux + d1.y * uy + d2.x * uz;
            fz = d1.x * ux + d2.x * uy + d2.y * uz;
         }
#pragma unroll
         for (int dx = 0; dx < D; dx++)
         {
            const double bq = b.B[qx + MQ * dx], gq = b.G[qx + MQ * dx];
            double t0 = T0[dx];
            if (MASS) { t0 += bq * m; }
            if (DIFF)
            {
               t0 += gq * fx;
               T1[dx] += bq * fy;
               T2[dx] += bq * fz;
            }
            T0[dx] = t0;
         }
      }
      // transpose: Yo += (B_y B_z) T0 + (G_y B_z) T1 + (B_y G_z) T2
#pragma unroll
      for (int dz = 0; dz < D; dz++)
#pragma unroll
         for (int dy = 0; dy < D; dy++)
         {
            const double p0 = P[0 * DD + dz * D + dy];
            const double p1 = P[1 * DD + dz * D + dy];
            const double p2 = P[2 * DD + dz * D + dy];
#pragma unroll
            for (int dx = 0; dx < D; dx++)
            {
               double yo = Yo[(dz * D + dy) * D + dx] + p0 * T0[dx];
               if (DIFF) { yo += p1 * T1[dx] + p2 * T2[dx]; }
               Yo[(dz * D + dy) * D + dx] = yo;
            }
         }
   }

   // ---- scatter (ElementRestriction::MultTranspose) by FP64 atomics ----
   if (active)
   {
#pragma unroll
      for (int a = 0; a < ND; a++)
      {
         const int g = mp[a * 64];
         const int d = bdof(g);
         double *dst = (!SPLIT || d < n_owned) ? y + d : yg + (d - n_owned);
         unsafeAtomicAdd(dst, bneg(g) ? -Yo[a] : Yo[a]);
      }
   }
}

// Software-pipelined variant: the 27 gathered dofs live in LDS (a private [a][lane]
// slot per wave: conflict-free ds_read_b64), which frees the VGPRs to hold the NEXT
// row's qdata in flight while the current row is computed (double buffering).
// VAR bit0: plain stores instead of atomics (diagnostic: atomic cost, wrong result)
// VAR bit1: default-policy (not nontemporal) qdata loads
// XCD-aware workgroup order: the hardware deals workgroup i to XCD i % 8 (MI355X_MICROARCH.md,
// "Workgroup dispatch"); remapping i to a contiguous range per XCD keeps neighbouring bricks
// (which share x values) in one XCD's L2.  A bijection on [0, G) for any G.
__device__ __forceinline__ int xcd_contiguous(int i, int G)
{
   const int q = G >> 3, r = G & 7, x = i & 7, j = i >> 3;
   return x * q + (x < r ? x : r) + j;
}

// In-wave assembly of a thread-per-element block's outputs and their store (apply and
// diagonal kernels).  A 4x4x4 brick is one wave: x, y, z neighbours are lanes +1, +4, +16;
// setup-computed lane flags say which faces really coincide (dof-index equality), so any
// element order is correct; bricks make it effective.  SIGNS: apply the map's orientation
// signs before summation (y = A x; the diagonal's signs square away).  Then entries whose
// face was sent away hold nothing; a dof held once in the whole mesh is plain-stored; a
// shared one goes to its dense partial slot [blk][a][lane] (summed in a fixed order by
// k_sum_partials: deterministic, no atomics, no y memset) or, without a partial buffer, is
// atomically added.  PLAIN: diagnostic (plain stores only; wrong for shared dofs).
// Rows per wave of the LDS region the cross-wave face exchange uses (3 faces of D x D).
template <int D>
struct XwaveRows
{
   static constexpr int ND = D * D * D, R = ND > 3 * D * D ? ND : 3 * D * D;
};

// XW: after each direction's in-wave merge, faces shared with another wave of the workgroup
// (lane flags 64|128|256 + the sending wave in bits 9-17, see build_merge_plan) move through
// LDS: the sending lanes (low face, e_dir = 0) park their face in their own wave's region
// xb[w][XR][64] (the kernel's x staging area, no longer read), a barrier, the receiving lanes
// (high face, e_dir = 3) add it.  Every wave of the workgroup must call this (wave_on false:
// barriers only).
template <int D, bool SPLIT, bool SIGNS, bool PLAIN, bool XW = false>
__device__ __forceinline__ void tpe_assemble_store(double (&Yo)[D * D * D], const int *__restrict__ mp, int fl,
                                                   int blk, int lane, bool active, int n_owned,
                                                   double *__restrict__ y, double *__restrict__ yg,
                                                   double *__restrict__ part, const int *__restrict__ pslot,
                                                   double *xb = nullptr, int w = 0, bool wave_on = true)
{
   constexpr int ND = D * D * D, XR = XwaveRows<D>::R;
   if (SIGNS && wave_on)
   {
#pragma unroll
      for (int a = 0; a < ND; a++)
      {
         if (bneg(mp[a * 64])) { Yo[a] = -Yo[a]; }
      }
   }
   auto merge = [&](int dir, int delta, int recv_bit, int sent_bit, auto face) {
      if (XW && wave_on && ((lane / delta) & 3) == 0 && (fl & sent_bit))
      {
#pragma unroll
         for (int j = 0; j < D; j++)
#pragma unroll
            for (int i = 0; i < D; i++) { xb[((w * XR) + dir * D * D + j * D + i) * 64 + lane] = Yo[face(0, i, j)]; }
      }
      if (wave_on)
      {
#pragma unroll
         for (int j = 0; j < D; j++)
#pragma unroll
            for (int i = 0; i < D; i++)
            {
               const double v = __shfl_down(Yo[face(0, i, j)], delta, 64);
               if (fl & recv_bit) { Yo[face(D - 1, i, j)] += v; }
               if (fl & sent_bit) { Yo[face(0, i, j)] = 0.0; }
            }
      }
      if (XW)
      {
         __syncthreads();
         if (wave_on && (fl & (64 << dir)))
         {
            const int pw = (fl >> (9 + 3 * dir)) & 7;
#pragma unroll
            for (int j = 0; j < D; j++)
#pragma unroll
               for (int i = 0; i < D; i++)
               {
                  Yo[face(D - 1, i, j)] += xb[((pw * XR) + dir * D * D + j * D + i) * 64 + lane - 3 * delta];
               }
         }
      }
   };
   merge(0, 1, 1, 2, [](int s, int i, int j) { return (j * D + i) * D + s; });    // x: (dz=j, dy=i)
   merge(1, 4, 4, 8, [](int s, int i, int j) { return (j * D + s) * D + i; });    // y: (dz=j, dx=i)
   merge(2, 16, 16, 32, [](int s, int i, int j) { return (s * D + j) * D + i; }); // z: (dy=j, dx=i)
   if (!active || !wave_on) { return; }
   const bool sx = fl & 2, sy = fl & 8, sz = fl & 32;
#pragma unroll
   for (int dz = 0; dz < D; dz++)
#pragma unroll
      for (int dy = 0; dy < D; dy++)
#pragma unroll
         for (int dx = 0; dx < D; dx++)
         {
            if ((dx == 0 && sx) || (dy == 0 && sy) || (dz == 0 && sz)) { continue; }
            const int a = (dz * D + dy) * D + dx;
            const int g = mp[a * 64];
            const int d = bdof(g);
            double *dst = (!SPLIT || d < n_owned) ? y + d : yg + (d - n_owned);
            if (!bshared(g) || PLAIN) { *dst = Yo[a]; }
            else if (part)
            {
               // pslot: the entry's position in its dof's contiguous run (summation pass reads
               // each dof's holders contiguously); else the dense [blk][a][lane] slot
               const size_t ent = ((size_t)blk * ND + a) * 64 + lane;
               part[pslot ? (size_t)pslot[ent] : ent] = Yo[a];
            }
            else { unsafeAtomicAdd(dst, Yo[a]); }
         }
}

// AFF: AFFINE qdata (kernels.hpp): the element's C is loaded once, each quadrature point
// streams one 16-byte pair (W beta, W alpha det J) instead of four loads of 56 bytes.
template <int D, int Q, bool MASS, bool DIFF, bool SPLIT, int VAR, bool AFF = false>
__global__ void __launch_bounds__(256, (VAR & 8) ? 2 : 1)
k_apply_tpe_pf(int ne, int blk_begin, int blk_end, int n_owned, const int *__restrict__ gmap,
               const double *__restrict__ qdd, const double *__restrict__ qdm,
               const double *__restrict__ x, const double *__restrict__ xg,
               double *__restrict__ y, double *__restrict__ yg, const Basis1D b,
               const double *__restrict__ rowtab, const int *__restrict__ lane_flags,
               double *__restrict__ part, const int *__restrict__ pslot)
{
   constexpr int ND = D * D * D, NQ = Q * Q * Q, NQH = (NQ + 1) / 2, DD = D * D;
   constexpr int NR = Q * Q;  // rows
   __shared__ double sX[4][ND][64];
   const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
   const int wg = (VAR & 16) ? xcd_contiguous(blockIdx.x, gridDim.x) : (int)blockIdx.x;
   const int blk = blk_begin + wg * 4 + w;
   if (blk >= blk_end) { return; }  // wave-uniform; no block-wide barrier below
   const int e = blk * 64 + lane;
   const bool active = e < ne;
   const int *mp = gmap + (size_t)blk * ND * 64 + lane;
#pragma unroll
   for (int a = 0; a < ND; a++)
   {
      const int g = mp[a * 64];
      const int d = bdof(g);
      const double v = (!SPLIT || d < n_owned) ? x[d] : xg[d - n_owned];
      sX[w][a][lane] = bneg(g) ? -v : v;
   }
   double Yo[ND];
#pragma unroll
   for (int a = 0; a < ND; a++) { Yo[a] = 0.0; }

   const double *qd = qdd + (size_t)blk * NQ * 3 * 128 + lane * 2;
   const double *qm = qdm + (size_t)blk * NQH * 128 + lane * 2;
   auto ld2 = [&](const double *p) -> v2d {
      if (VAR & 2) { return *reinterpret_cast<const v2d *>(p); }
      return __builtin_nontemporal_load(reinterpret_cast<const v2d *>(p));
   };
   // row buffers: diffusion pairs (3 per point) and mass values (Q per row); AFF: one
   // (W beta, W alpha det J) pair per point and the element's C in registers
   v2d cd[Q][3], nd_[Q][3];
   double cm[Q], nm[Q];
   v2d ca[Q], na[Q], ce[3];
   const double *qa = qdm + (size_t)blk * NQ * 128 + lane * 2;
   if (AFF)
   {
      const double *qc = qdd + (size_t)blk * 3 * 128 + lane * 2;
#pragma unroll
      for (int k = 0; k < 3; k++) { ce[k] = ld2(qc + k * 128); }
   }
   auto load_row = [&](int row, v2d (&dq)[Q][3], double (&mq)[Q], v2d (&aq)[Q]) {
#pragma unroll
      for (int qx = 0; qx < Q; qx++)
      {
         const int q = row * Q + qx;
         if (AFF)
         {
            aq[qx] = ld2(qa + (size_t)q * 128);
            continue;
         }
         if (DIFF)
         {
#pragma unroll
            for (int k = 0; k < 3; k++) { dq[qx][k] = ld2(qd + ((size_t)q * 3 + k) * 128); }
         }
         if (MASS) { mq[qx] = qm[(size_t)(q >> 1) * 128 + (q & 1)]; }
      }
   };
   load_row(0, cd, cm, ca);

#pragma unroll 1
   for (int row = 0; row < NR; row++)
   {
      if (row + 1 < NR) { load_row(row + 1, nd_, nm, na); }
      const double *P = rowtab + (size_t)row * 3 * DD;
      double Y00[D], Y01[D], Y10[D];
#pragma unroll
      for (int dx = 0; dx < D; dx++)
      {
         double u = 0.0, v = 0.0, wv = 0.0;
#pragma unroll
         for (int dz = 0; dz < D; dz++)
#pragma unroll
            for (int dy = 0; dy < D; dy++)
            {
               const double c = sX[w][(dz * D + dy) * D + dx][lane];
               u += P[0 * DD + dz * D + dy] * c;
               if (DIFF)
               {
                  v += P[1 * DD + dz * D + dy] * c;
                  wv += P[2 * DD + dz * D + dy] * c;
               }
            }
         Y00[dx] = u; Y01[dx] = v; Y10[dx] = wv;
      }
      double T0[D], T1[D], T2[D];
#pragma unroll
      for (int dx = 0; dx < D; dx++) { T0[dx] = 0.0; T1[dx] = 0.0; T2[dx] = 0.0; }
#pragma unroll
      for (int qx = 0; qx < Q; qx++)
      {
         double u = 0.0, ux = 0.0, uy = 0.0, uz = 0.0;
#pragma unroll
         for (int dx = 0; dx < D; dx++)
         {
            const double bq = b.B[qx + MQ * dx], gq = b.G[qx + MQ * dx];
            if (MASS) { u += bq * Y00[dx]; }
            if (DIFF)
            {
               ux += gq * Y00[dx];
               uy += bq * Y01[dx];
               uz += bq * Y10[dx];
            }
         }
         double m = 0.0, fx = 0.0, fy = 0.0, fz = 0.0;
         if (AFF)
         {
            const v2d sa = ca[qx];
            m = sa.y * u;
            fx = sa.x * (ce[0].x * ux + ce[0].y * uy + ce[1].x * uz);
            fy = sa.x * (ce[0].y * ux + ce[1].y * uy + ce[2].x * uz);
            fz = sa.x * (ce[1].x * ux + ce[2].x * uy + ce[2].y * uz);
         }
         else
         {
         if (MASS) { m = cm[qx] * u; }
         if (DIFF)
         {
            const v2d d0 = cd[qx][0], d1 = cd[qx][1], d2 = cd[qx][2];
            fx = d0.x * ux + d0.y * uy + d1.x * uz;
            fy = d0.y * ux + d1.y * uy + d2.x * uz;
            fz = d1.x * ux + d2.x * uy + d2.y * uz;
         }
         }
#pragma unroll
         for (int dx = 0; dx < D; dx++)
         {
            const double bq = b.B[qx + MQ * dx], gq = b.G[qx + MQ * dx];
            double t0 = T0[dx];
            if (MASS) { t0 += bq * m; }
            if (DIFF)
            {
               t0 += gq * fx;
               T1[dx] += bq * fy;
               T2[dx] += bq * fz;
            }
            T0[dx] = t0;
         }
      }
#pragma unroll
      for (int dz = 0; dz < D; dz++)
#pragma unroll
         for (int dy = 0; dy < D; dy++)
         {
            const double p0 = P[0 * DD + dz * D + dy];
            const double p1 = P[1 * DD + dz * D + dy];
            const double p2 = P[2 * DD + dz * D + dy];
#pragma unroll
            for (int dx = 0; dx < D; dx++)
            {
               double yo = Yo[(dz * D + dy) * D + dx] + p0 * T0[dx];
               if (DIFF) { yo += p1 * T1[dx] + p2 * T2[dx]; }
               Yo[(dz * D + dy) * D + dx] = yo;
            }
         }
#pragma unroll
      for (int qx = 0; qx < Q; qx++)
      {
#pragma unroll
         for (int k = 0; k < 3; k++) { cd[qx][k] = nd_[qx][k]; }
         cm[qx] = nm[qx];
         ca[qx] = na[qx];
      }
   }
   tpe_assemble_store<D, SPLIT, true, (VAR & 1) != 0>(Yo, mp, lane_flags[(size_t)blk * 64 + lane], blk, lane, active,
                                                      n_owned, y, yg, part, pslot);
}

// Thread-per-element apply on AFFINE qdata, sum-factorised per quadrature plane qz: the
// x-values (LDS) are contracted in z once per plane (ZB = B_z X, ZG = G_z X, D^2 each), each of
// the plane's Q rows contracts them in y (3 D^2 multiply-adds instead of the row kernel's
// 3 D^3 on precomputed B_y B_z products), then x / weighting / x-transpose as in
// k_apply_tpe_pf; the row's y-transpose accumulates into the plane sums SB, SG (2 D^2 + D^2)
// and the plane ends with one z-transpose into the element outputs (2 D^3).  At p = 2 that is
// 229 instead of 310 FP64 multiply-adds per row (-26%).  Same gather, row prefetch,
// in-wave face assembly and deterministic store as k_apply_tpe_pf.
// VAR & 128: workgroups of 8 waves (2 x 2 x 2 bricks share faces through LDS; 110 KB of LDS at
// p = 2, one workgroup per CU) instead of 4.
template <int D, int Q, bool SPLIT, int VAR>
__global__ void __launch_bounds__((VAR & 128) ? 512 : 256, (VAR & 8) ? 2 : 1)
k_apply_tpe_sf(int ne, int blk_begin, int blk_end, int n_owned, const int *__restrict__ gmap,
               const double *__restrict__ qdd, const double *__restrict__ qdm,
               const double *__restrict__ x, const double *__restrict__ xg,
               double *__restrict__ y, double *__restrict__ yg, const Basis1D b,
               const int *__restrict__ lane_flags, double *__restrict__ part, const int *__restrict__ pslot)
{
   constexpr int ND = D * D * D, NQ = Q * Q * Q, NR = Q * Q, XR = XwaveRows<D>::R, WPG = (VAR & 128) ? 8 : 4;
   __shared__ double sX[WPG][XR][64];  // gathered x; then the cross-wave face exchange
   const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
   const int blk = blk_begin + (int)blockIdx.x * WPG + w;
   const bool wave_on = blk < blk_end;  // wave-uniform; every wave reaches the store's barriers
   const int e = blk * 64 + lane;
   const bool active = wave_on && e < ne;
   const int *mp = gmap + (size_t)blk * ND * 64 + lane;
   double Yo[ND];
#pragma unroll
   for (int a = 0; a < ND; a++) { Yo[a] = 0.0; }
   if (wave_on)
   {
#pragma unroll
   for (int a = 0; a < ND; a++)
   {
      const int g = mp[a * 64];
      const int d = bdof(g);
      const double v = (!SPLIT || d < n_owned) ? x[d] : xg[d - n_owned];
      sX[w][a][lane] = bneg(g) ? -v : v;
   }
   auto ld2 = [&](const double *p) -> v2d {
      if (VAR & 2) { return *reinterpret_cast<const v2d *>(p); }
      return __builtin_nontemporal_load(reinterpret_cast<const v2d *>(p));
   };
   v2d ce[3];
   {
      const double *qc = qdd + (size_t)blk * 3 * 128 + lane * 2;
#pragma unroll
      for (int k = 0; k < 3; k++) { ce[k] = ld2(qc + k * 128); }
   }
   const double *qa = qdm + (size_t)blk * NQ * 128 + lane * 2;
   // VAR & 4: rows prefetched two ahead (8 KiB per wave in flight instead of 4)
   constexpr bool DEEP = (VAR & 4) != 0;
   // VAR & 32: a whole plane prefetched (rows of plane qz + 1 in flight while plane qz
   // computes: 16 KiB per wave), for one wave per SIMD with the AGPRs as the ring
   constexpr bool PLANE = (VAR & 32) != 0;
   v2d ca[Q], na[Q], n2[Q], pb[Q][Q];
   auto load_row = [&](int row, v2d (&aq)[Q]) {
#pragma unroll
      for (int qx = 0; qx < Q; qx++) { aq[qx] = ld2(qa + (size_t)(row * Q + qx) * 128); }
   };
   if (PLANE)
   {
#pragma unroll
      for (int qy = 0; qy < Q; qy++) { load_row(qy, pb[qy]); }
   }
   else { load_row(0, ca); }
   if (DEEP) { load_row(1, na); }

#pragma unroll 1
   for (int qz = 0; qz < Q; qz++)
   {
      double bz[D], gz[D];
#pragma unroll
      for (int dz = 0; dz < D; dz++) { bz[dz] = b.B[qz + MQ * dz]; gz[dz] = b.G[qz + MQ * dz]; }
      // opaque lane index: the plane re-reads X from LDS instead of keeping 27 values live
      int ll = lane;
      asm volatile("" : "+v"(ll));
      double ZB[D][D], ZG[D][D], SB[D][D], SG[D][D];
#pragma unroll
      for (int dy = 0; dy < D; dy++)
#pragma unroll
         for (int dx = 0; dx < D; dx++)
         {
            double zb = 0.0, zg = 0.0;
#pragma unroll
            for (int dz = 0; dz < D; dz++)
            {
               const double c = sX[w][(dz * D + dy) * D + dx][ll];
               zb += bz[dz] * c;
               zg += gz[dz] * c;
            }
            ZB[dy][dx] = zb; ZG[dy][dx] = zg;
            SB[dy][dx] = 0.0; SG[dy][dx] = 0.0;
         }
      // one row (qz, qy) of Q points: y-forward, x-forward, weighting, x-transpose, y-transpose
      auto row_body = [&](int qy, const v2d (&cur)[Q]) {
         double Y00[D], Y01[D], Y10[D];
#pragma unroll
         for (int dx = 0; dx < D; dx++)
         {
            double u = 0.0, v = 0.0, wv = 0.0;
#pragma unroll
            for (int dy = 0; dy < D; dy++)
            {
               const double by = b.B[qy + MQ * dy], gy = b.G[qy + MQ * dy];
               u += by * ZB[dy][dx];
               v += gy * ZB[dy][dx];
               wv += by * ZG[dy][dx];
            }
            Y00[dx] = u; Y01[dx] = v; Y10[dx] = wv;
         }
         double T0[D], T1[D], T2[D];
#pragma unroll
         for (int dx = 0; dx < D; dx++) { T0[dx] = 0.0; T1[dx] = 0.0; T2[dx] = 0.0; }
#pragma unroll
         for (int qx = 0; qx < Q; qx++)
         {
            double u = 0.0, ux = 0.0, uy = 0.0, uz = 0.0;
#pragma unroll
            for (int dx = 0; dx < D; dx++)
            {
               const double bq = b.B[qx + MQ * dx], gq = b.G[qx + MQ * dx];
               u += bq * Y00[dx];
               ux += gq * Y00[dx];
               uy += bq * Y01[dx];
               uz += bq * Y10[dx];
            }
            const v2d sa = cur[qx];
            const double m = sa.y * u;
            const double fx = sa.x * (ce[0].x * ux + ce[0].y * uy + ce[1].x * uz);
            const double fy = sa.x * (ce[0].y * ux + ce[1].y * uy + ce[2].x * uz);
            const double fz = sa.x * (ce[1].x * ux + ce[2].x * uy + ce[2].y * uz);
#pragma unroll
            for (int dx = 0; dx < D; dx++)
            {
               const double bq = b.B[qx + MQ * dx], gq = b.G[qx + MQ * dx];
               T0[dx] += bq * m + gq * fx;
               T1[dx] += bq * fy;
               T2[dx] += bq * fz;
            }
         }
#pragma unroll
         for (int dy = 0; dy < D; dy++)
         {
            const double by = b.B[qy + MQ * dy], gy = b.G[qy + MQ * dy];
#pragma unroll
            for (int dx = 0; dx < D; dx++)
            {
               SB[dy][dx] += by * T0[dx] + gy * T1[dx];
               SG[dy][dx] += by * T2[dx];
            }
         }
      };
      if constexpr (PLANE)
      {
         // the plane's rows are in pb (loaded during the previous plane); each row's
         // buffer is refilled with the next plane's row right after use
#pragma unroll
         for (int qy = 0; qy < Q; qy++)
         {
            row_body(qy, pb[qy]);
            if (qz + 1 < Q) { load_row((qz + 1) * Q + qy, pb[qy]); }
         }
      }
      else
      {
#pragma unroll 1
      for (int qy = 0; qy < Q; qy++)
      {
         const int row = qz * Q + qy;
         if (DEEP) { if (row + 2 < NR) { load_row(row + 2, n2); } }
         else if (row + 1 < NR) { load_row(row + 1, na); }
         row_body(qy, ca);
#pragma unroll
         for (int qx = 0; qx < Q; qx++)
         {
            ca[qx] = na[qx];
            if (DEEP) { na[qx] = n2[qx]; }
         }
      }
      }
#pragma unroll
      for (int dz = 0; dz < D; dz++)
#pragma unroll
         for (int dy = 0; dy < D; dy++)
#pragma unroll
            for (int dx = 0; dx < D; dx++)
            {
               Yo[(dz * D + dy) * D + dx] += bz[dz] * SB[dy][dx] + gz[dz] * SG[dy][dx];
            }
   }
   }  // wave_on
   tpe_assemble_store<D, SPLIT, true, (VAR & 1) != 0, true>(Yo, mp, wave_on ? lane_flags[(size_t)blk * 64 + lane] : 0,
                                                            blk, lane, active, n_owned, y, yg, part, pslot,
                                                            &sX[0][0][0], w, wave_on);
}

// Latency variant of k_apply_tpe_sf for small block ranges (the distributed Mult's boundary
// elements, on the critical path of the exchange): one workgroup per 64-element block, its
// four waves gather the x-values together and take one quadrature plane each (all of the
// plane's pairs loaded up front), so a block costs one plane's latency instead of four.
// Waves 1..3 hand their partial outputs to wave 0 through LDS, which adds them in a fixed
// order (deterministic) and assembles / stores exactly like k_apply_tpe_sf.
template <int D, int Q, bool SPLIT>
__global__ void __launch_bounds__(256)
k_apply_tpe_pp(int ne, int blk_begin, int n_owned, const int *__restrict__ gmap,
               const double *__restrict__ qdd, const double *__restrict__ qdm,
               const double *__restrict__ x, const double *__restrict__ xg,
               double *__restrict__ y, double *__restrict__ yg, const Basis1D b,
               const int *__restrict__ lane_flags, double *__restrict__ part, const int *__restrict__ pslot)
{
   static_assert(Q <= 4, "one plane per wave");
   constexpr int ND = D * D * D, NQ = Q * Q * Q;
   __shared__ double sX[ND][64];
   __shared__ double sY[3][ND][64];
   const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
   const int blk = blk_begin + (int)blockIdx.x;
   const int e = blk * 64 + lane;
   const bool active = e < ne;
   const int *mp = gmap + (size_t)blk * ND * 64 + lane;
   for (int a = w; a < ND; a += 4)
   {
      const int g = mp[a * 64];
      const int d = bdof(g);
      const double v = (!SPLIT || d < n_owned) ? x[d] : xg[d - n_owned];
      sX[a][lane] = bneg(g) ? -v : v;
   }
   double Yo[ND];
#pragma unroll
   for (int a = 0; a < ND; a++) { Yo[a] = 0.0; }
   const int qz = w;
   v2d ce[3], pr[Q][Q];
   if (qz < Q)
   {
      const double *qc = qdd + (size_t)blk * 3 * 128 + lane * 2;
#pragma unroll
      for (int k = 0; k < 3; k++) { ce[k] = *reinterpret_cast<const v2d *>(qc + k * 128); }
      const double *qa = qdm + (size_t)blk * NQ * 128 + lane * 2;
#pragma unroll
      for (int qy = 0; qy < Q; qy++)
#pragma unroll
         for (int qx = 0; qx < Q; qx++)
         {
            pr[qy][qx] = __builtin_nontemporal_load(
               reinterpret_cast<const v2d *>(qa + (size_t)((qz * Q + qy) * Q + qx) * 128));
         }
   }
   __syncthreads();
   if (qz < Q)
   {
      double bz[D], gz[D];
#pragma unroll
      for (int dz = 0; dz < D; dz++) { bz[dz] = b.B[qz + MQ * dz]; gz[dz] = b.G[qz + MQ * dz]; }
      double ZB[D][D], ZG[D][D], SB[D][D], SG[D][D];
#pragma unroll
      for (int dy = 0; dy < D; dy++)
#pragma unroll
         for (int dx = 0; dx < D; dx++)
         {
            double zb = 0.0, zg = 0.0;
#pragma unroll
            for (int dz = 0; dz < D; dz++)
            {
               const double c = sX[(dz * D + dy) * D + dx][lane];
               zb += bz[dz] * c;
               zg += gz[dz] * c;
            }
            ZB[dy][dx] = zb; ZG[dy][dx] = zg;
            SB[dy][dx] = 0.0; SG[dy][dx] = 0.0;
         }
#pragma unroll
      for (int qy = 0; qy < Q; qy++)
      {
         double Y00[D], Y01[D], Y10[D];
#pragma unroll
         for (int dx = 0; dx < D; dx++)
         {
            double u = 0.0, v = 0.0, wv = 0.0;
#pragma unroll
            for (int dy = 0; dy < D; dy++)
            {
               const double by = b.B[qy + MQ * dy], gy = b.G[qy + MQ * dy];
               u += by * ZB[dy][dx];
               v += gy * ZB[dy][dx];
               wv += by * ZG[dy][dx];
            }
            Y00[dx] = u; Y01[dx] = v; Y10[dx] = wv;
         }
         double T0[D], T1[D], T2[D];
#pragma unroll
         for (int dx = 0; dx < D; dx++) { T0[dx] = 0.0; T1[dx] = 0.0; T2[dx] = 0.0; }
#pragma unroll
         for (int qx = 0; qx < Q; qx++)
         {
            double u = 0.0, ux = 0.0, uy = 0.0, uz = 0.0;
#pragma unroll
            for (int dx = 0; dx < D; dx++)
            {
               const double bq = b.B[qx + MQ * dx], gq = b.G[qx + MQ * dx];
               u += bq * Y00[dx];
               ux += gq * Y00[dx];
               uy += bq * Y01[dx];
               uz += bq * Y10[dx];
            }
            const v2d sa = pr[qy][qx];
            const double m = sa.y * u;
            const double fx = sa.x * (ce[0].x * ux + ce[0].y * uy + ce[1].x * uz);
            const double fy = sa.x * (ce[0].y * ux + ce[1].y * uy + ce[2].x * uz);
            const double fz = sa.x * (ce[1].x * ux + ce[2].x * uy + ce[2].y * uz);
#pragma unroll
            for (int dx = 0; dx < D; dx++)
            {
               const double bq = b.B[qx + MQ * dx], gq = b.G[qx + MQ * dx];
               T0[dx] += bq * m + gq * fx;
               T1[dx] += bq * fy;
               T2[dx] += bq * fz;
            }
         }
#pragma unroll
         for (int dy = 0; dy < D; dy++)
         {
            const double by = b.B[qy + MQ * dy], gy = b.G[qy + MQ * dy];
#pragma unroll
            for (int dx = 0; dx < D; dx++)
            {
               SB[dy][dx] += by * T0[dx] + gy * T1[dx];
               SG[dy][dx] += by * T2[dx];
            }
         }
      }
#pragma unroll
      for (int dz = 0; dz < D; dz++)
#pragma unroll
         for (int dy = 0; dy < D; dy++)
#pragma unroll
            for (int dx = 0; dx < D; dx++)
            {
               Yo[(dz * D + dy) * D + dx] = bz[dz] * SB[dy][dx] + gz[dz] * SG[dy][dx];
            }
   }
   if (w > 0)
   {
#pragma unroll
      for (int a = 0; a < ND; a++) { sY[w - 1][a][lane] = Yo[a]; }
   }
   __syncthreads();
   if (w != 0) { return; }
#pragma unroll
   for (int k = 0; k < 3; k++)
#pragma unroll
      for (int a = 0; a < ND; a++) { Yo[a] += sY[k][a][lane]; }
   tpe_assemble_store<D, SPLIT, true, false>(Yo, mp, lane_flags[(size_t)blk * 64 + lane], blk, lane, active,
                                             n_owned, y, yg, part, pslot);
}

// PA diagonal, thread per element on the blocked layout (PADiffusionDiagonal3D and the
// mass diagonal, bilininteg_diffusion_kernels.hpp:369, bilininteg_mass_kernels.hpp:325,
// assembled like AssembleDiagonal's E->L transpose, bilinearform_ext.cpp:370-454):
//   diag(a) = sum_q grad(phi_a)^T O_q grad(phi_a) + m_q phi_a^2,  phi_a = B_x B_y B_z,
// sum-factorised per quadrature row (qy, qz): seven x-contractions S_k(dx) of the row's
// qdata, then the (dy, dz) factors of the row from a table, [6][dz][dy] = (By Bz)^2,
// (Gy Bz)^2, (By Gz)^2, Gy By Bz^2, By^2 Gz Bz, Gy By Gz Bz.  Output assembled and stored
// exactly like k_apply_tpe_pf's (in-wave faces, plain stores, partial slots): every
// diagonal entry written once, deterministic, no memset.
template <int D, int Q, bool MASS, bool DIFF, bool SPLIT, bool AFF = false, int WPG = 4>
__global__ void __launch_bounds__(64 * WPG)
k_diag_tpe(int ne, int blk_begin, int blk_end, int n_owned, const int *__restrict__ gmap,
           const double *__restrict__ qdd, const double *__restrict__ qdm, double *__restrict__ y,
           double *__restrict__ yg, const Basis1D b, const double *__restrict__ drow,
           const int *__restrict__ lane_flags, double *__restrict__ part, const int *__restrict__ pslot)
{
   constexpr int ND = D * D * D, NQ = Q * Q * Q, NQH = (NQ + 1) / 2, DD = D * D, XR = XwaveRows<D>::R;
   __shared__ double xb[AFF ? WPG * XR * 64 : 1];  // AFF: cross-wave face exchange (as the apply's plan)
   const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
   const int blk = blk_begin + blockIdx.x * WPG + w;
   const bool wave_on = blk < blk_end;  // wave-uniform
   if (!AFF && !wave_on) { return; }    // no block-wide barrier without AFF
   const bool active = wave_on && blk * 64 + lane < ne;
   const int *mp = gmap + (size_t)blk * ND * 64 + lane;
   const double *qd = qdd + (size_t)blk * NQ * 3 * 128 + lane * 2;
   const double *qm = qdm + (size_t)blk * NQH * 128 + lane * 2;
   const double *qa = qdm + (size_t)blk * NQ * 128 + lane * 2;  // AFF pairs
   v2d ce[3];
   if (AFF && wave_on)
   {
#pragma unroll
      for (int k = 0; k < 3; k++) { ce[k] = *reinterpret_cast<const v2d *>(qdd + (size_t)blk * 3 * 128 + lane * 2 + k * 128); }
   }
   double Yo[ND];
#pragma unroll
   for (int a = 0; a < ND; a++) { Yo[a] = 0.0; }
#pragma unroll 1
   for (int row = 0; row < (wave_on ? Q * Q : 0); row++)
   {
      double S[7][D];
#pragma unroll
      for (int k = 0; k < 7; k++)
#pragma unroll
         for (int dx = 0; dx < D; dx++) { S[k][dx] = 0.0; }
#pragma unroll
      for (int qx = 0; qx < Q; qx++)
      {
         const int q = row * Q + qx;
         v2d d0 = {0.0, 0.0}, d1 = {0.0, 0.0}, d2 = {0.0, 0.0};
         double m = 0.0;
         if (AFF)
         {
            const v2d sa = *reinterpret_cast<const v2d *>(qa + (size_t)q * 128);
            d0 = sa.x * ce[0];
            d1 = sa.x * ce[1];
            d2 = sa.x * ce[2];
            m = sa.y;
         }
         else
         {
         if (DIFF)
         {
            d0 = *reinterpret_cast<const v2d *>(qd + ((size_t)q * 3 + 0) * 128);
            d1 = *reinterpret_cast<const v2d *>(qd + ((size_t)q * 3 + 1) * 128);
            d2 = *reinterpret_cast<const v2d *>(qd + ((size_t)q * 3 + 2) * 128);
         }
         if (MASS) { m = qm[(size_t)(q >> 1) * 128 + (q & 1)]; }
         }
#pragma unroll
         for (int dx = 0; dx < D; dx++)
         {
            const double bx = b.B[qx + MQ * dx], gx = b.G[qx + MQ * dx];
            const double bb = bx * bx, gb = gx * bx;
            if (DIFF)
            {
               S[0][dx] += gx * gx * d0.x;  // O11
               S[1][dx] += bb * d1.y;       // O22
               S[2][dx] += bb * d2.y;       // O33
               S[3][dx] += gb * d0.y;       // O12
               S[4][dx] += gb * d1.x;       // O13
               S[5][dx] += bb * d2.x;       // O23
            }
            if (MASS) { S[6][dx] += bb * m; }
         }
      }
      const double *P = drow + (size_t)row * 6 * DD;
#pragma unroll
      for (int dz = 0; dz < D; dz++)
#pragma unroll
         for (int dy = 0; dy < D; dy++)
         {
            const int o = dz * D + dy;
            const double p0 = P[o], p1 = P[DD + o], p2 = P[2 * DD + o];
            const double p3 = P[3 * DD + o], p4 = P[4 * DD + o], p5 = P[5 * DD + o];
#pragma unroll
            for (int dx = 0; dx < D; dx++)
            {
               double v = p0 * (S[0][dx] + S[6][dx]) + p1 * S[1][dx] + p2 * S[2][dx];
               v += 2.0 * (p3 * S[3][dx] + p4 * S[4][dx] + p5 * S[5][dx]);
               Yo[o * D + dx] += v;
            }
         }
   }
   tpe_assemble_store<D, SPLIT, false, false, AFF>(Yo, mp, wave_on ? lane_flags[(size_t)blk * 64 + lane] : 0, blk,
                                                    lane, active, n_owned, y, yg, part, pslot, xb, w, wave_on);
}

// --------------------------------------------------------------------------
// Workgroup per element (lane per quadrature point), any layout, L- or E-vectors
// --------------------------------------------------------------------------

template <int D, int Q, bool MASS, bool DIFF, bool IN_E, bool OUT_E>
__global__ void k_apply_wpe(const int *__restrict__ pos, int kind, int ne, int e_begin, int n_owned,
                            const int *__restrict__ gmap,
                            const double *__restrict__ qdd, const double *__restrict__ qdm,
                            const double *__restrict__ x, const double *__restrict__ xg,
                            double *__restrict__ y, double *__restrict__ yg, const Basis1D b, int var)
{
   constexpr int ND = D * D * D, NQ = Q * Q * Q;
   // experiment knob (ECM2_WPE_VARIANT): bit 1 = plain stores (diagnostic, wrong y),
   // bit 2 = prefetch this thread's qdata before the contraction stages
   double pq[7];
   if ((var & 2) && threadIdx.x < NQ)
   {
      const int e = e_begin + blockIdx.x, t = threadIdx.x;
      if (MASS) { pq[6] = qd_mass_at(qdm, pos, kind, NQ, e, t); }
      if (DIFF)
      {
#pragma unroll
         for (int c = 0; c < 6; c++) { pq[c] = qd_diff_at(qdd, qdm, pos, kind, NQ, e, c, t); }
      }
   }
   __shared__ double sB[Q * D], sG[Q * D];
   __shared__ double sX[ND];
   __shared__ double s1a[D * D * Q], s1b[D * D * Q];
   __shared__ double s2a[D * Q * Q], s2b[D * Q * Q], s2c[D * Q * Q];
   __shared__ double s3m[NQ], s3x[NQ], s3y[NQ], s3z[NQ];
   __shared__ double s4a[Q * Q * D], s4b[Q * Q * D], s4c[Q * Q * D];
   __shared__ double s5a[Q * D * D], s5b[Q * D * D];
   const int e = e_begin + blockIdx.x;
   const int t = threadIdx.x;
   if (t < Q * D)
   {
      const int q = t % Q, d = t / Q;
      sB[q + Q * d] = b.B[q + MQ * d];
      sG[q + Q * d] = b.G[q + MQ * d];
   }
   if (t < ND)
   {
      if (IN_E) { sX[t] = x[(size_t)e * ND + t]; }
      else
      {
         const int g = gmap[(size_t)e * ND + t];
         const int d = dof_of(g);
         const double v = d < n_owned ? x[d] : xg[d - n_owned];
         sX[t] = g >= 0 ? v : -v;
      }
   }
   __syncthreads();
   // stage 1: x-contraction  (qx, dy, dz)
   if (t < D * D * Q)
   {
      const int qx = t % Q, dy = (t / Q) % D, dz = t / (Q * D);
      double u = 0.0, v = 0.0;
      for (int dx = 0; dx < D; dx++)
      {
         const double c = sX[(dz * D + dy) * D + dx];
         u += c * sB[qx + Q * dx];
         v += c * sG[qx + Q * dx];
      }
      s1a[t] = u;  // B_x
      s1b[t] = v;  // G_x
   }
   __syncthreads();
   // stage 2: y-contraction  (qx, qy, dz)
   if (t < D * Q * Q)
   {
      const int qx = t % Q, qy = (t / Q) % Q, dz = t / (Q * Q);
      double u = 0.0, v = 0.0, w = 0.0;
      for (int dy = 0; dy < D; dy++)
      {
         const int i = (dz * D + dy) * Q + qx;
         u += s1b[i] * sB[qy + Q * dy];   // G_x B_y
         v += s1a[i] * sG[qy + Q * dy];   // B_x G_y
         w += s1a[i] * sB[qy + Q * dy];   // B_x B_y
      }
      s2a[t] = u; s2b[t] = v; s2c[t] = w;
   }
   __syncthreads();
   // stage 3: z-contraction + pointwise qdata (qx, qy, qz)
   if (t < NQ)
   {
      const int qx = t % Q, qy = (t / Q) % Q, qz = t / (Q * Q);
      double gx = 0.0, gy = 0.0, gz = 0.0, u = 0.0;
      for (int dz = 0; dz < D; dz++)
      {
         const int i = (dz * Q + qy) * Q + qx;
         gx += s2a[i] * sB[qz + Q * dz];
         gy += s2b[i] * sB[qz + Q * dz];
         gz += s2c[i] * sG[qz + Q * dz];
         u += s2c[i] * sB[qz + Q * dz];
      }
      double m = 0.0, fx = 0.0, fy = 0.0, fz = 0.0;
      if (var & 2)
      {
         if (MASS) { m = pq[6] * u; }
         if (DIFF)
         {
            fx = (pq[0] * gx) + (pq[1] * gy) + (pq[2] * gz);
            fy = (pq[1] * gx) + (pq[3] * gy) + (pq[4] * gz);
            fz = (pq[2] * gx) + (pq[4] * gy) + (pq[5] * gz);
         }
      }
      else
      {
      if (MASS) { m = qd_mass_at(qdm, pos, kind, NQ, e, t) * u; }
      if (DIFF)
      {
         const double O11 = qd_diff_at(qdd, qdm, pos, kind, NQ, e, 0, t);
         const double O12 = qd_diff_at(qdd, qdm, pos, kind, NQ, e, 1, t);
         const double O13 = qd_diff_at(qdd, qdm, pos, kind, NQ, e, 2, t);
         const double O22 = qd_diff_at(qdd, qdm, pos, kind, NQ, e, 3, t);
         const double O23 = qd_diff_at(qdd, qdm, pos, kind, NQ, e, 4, t);
         const double O33 = qd_diff_at(qdd, qdm, pos, kind, NQ, e, 5, t);
         fx = (O11 * gx) + (O12 * gy) + (O13 * gz);
         fy = (O12 * gx) + (O22 * gy) + (O23 * gz);
         fz = (O13 * gx) + (O23 * gy) + (O33 * gz);
      }
      }
      s3m[t] = m; s3x[t] = fx; s3y[t] = fy; s3z[t] = fz;
   }
   __syncthreads();
   // stage 4: x-transpose (dx, qy, qz)
   if (t < Q * Q * D)
   {
      const int dx = t % D, qy = (t / D) % Q, qz = t / (D * Q);
      double u = 0.0, v = 0.0, w = 0.0;
      for (int qx = 0; qx < Q; qx++)
      {
         const int i = (qz * Q + qy) * Q + qx;
         u += s3x[i] * sG[qx + Q * dx] + s3m[i] * sB[qx + Q * dx];
         v += s3y[i] * sB[qx + Q * dx];
         w += s3z[i] * sB[qx + Q * dx];
      }
      s4a[t] = u; s4b[t] = v; s4c[t] = w;
   }
   __syncthreads();
   // stage 5: y-transpose (dx, dy, qz)
   if (t < Q * D * D)
   {
      const int dx = t % D, dy = (t / D) % D, qz = t / (D * D);
      double u = 0.0, w = 0.0;
      for (int qy = 0; qy < Q; qy++)
      {
         const int i = (qz * Q + qy) * D + dx;
         u += s4a[i] * sB[qy + Q * dy] + s4b[i] * sG[qy + Q * dy];
         w += s4c[i] * sB[qy + Q * dy];
      }
      s5a[t] = u; s5b[t] = w;
   }
   __syncthreads();
   // stage 6: z-transpose (dx, dy, dz) + output
   if (t < ND)
   {
      const int dx = t % D, dy = (t / D) % D, dz = t / (D * D);
      double u = 0.0;
      for (int qz = 0; qz < Q; qz++)
      {
         const int i = (qz * D + dy) * D + dx;
         u += s5a[i] * sB[qz + Q * dz] + s5b[i] * sG[qz + Q * dz];
      }
      if (OUT_E) { y[(size_t)e * ND + t] += u; }
      else
      {
         const int g = gmap[(size_t)e * ND + t];
         const int d = dof_of(g);
         double *dst = d < n_owned ? y + d : yg + (d - n_owned);
         if (var & 1) { *dst = g >= 0 ? u : -u; }
         else { unsafeAtomicAdd(dst, g >= 0 ? u : -u); }
      }
   }
}

// --------------------------------------------------------------------------
// Restriction, diagonal, vector kernels
// --------------------------------------------------------------------------

// --------------------------------------------------------------------------
// "Line" kernel: one wave per chunk of up to 8 x-adjacent elements, any (D, Q) with
// Q*Q <= 64 (p = 1..6), L-vectors in and out.  Each stage gives every active lane one
// 1D line of the current contraction direction in registers: a lane reads D (or Q)
// values from LDS once and produces Q (or D) outputs, so LDS traffic is one read per
// Q multiply-adds (the reference's smem kernels, bilininteg_diffusion_kernels.hpp:
// 989-1214, read two LDS operands per multiply-add).  B/G come from the kernel
// arguments (SGPR operands).  The z contraction, the quadrature-point weighting and
// the transposed z contraction are fused in registers on (qx, qy) lanes.
//   lanes (dy,dz): gather x-line, x-contract          -> s1 [2][dz][dy][qx]
//   lanes (qx,dz): y-contract                           -> s2 [3][dz][qy][qx]
//   lanes (qx,qy): z-contract, weight, z-transpose      -> s3 [3][dz][qy][qx]
//   lanes (qx,dz): y-transpose                          -> s4 [2][dz][dy][qx]
//   lanes (dy,dz): x-transpose, scatter
// Chunks: consecutive elements whose x-faces coincide (checked on the host).  Lane
// (dy,dz) holds entry (D-1,dy,dz) of element k and (0,dy,dz) of element k+1, so the
// shared face is summed in a register (carry) and only the last element stores it.
// The qdata registers are dead after the z stage: the next element's qdata is loaded
// into them there, overlapping its latency with the rest of this element.
// gmap: [e][ND] encoded dof | shared << 30 | sign << 31 (see PAForm::assemble);
// chunks[c] = first element | count << 24 (count <= 8).
// --------------------------------------------------------------------------
// Basis tables in constant memory, one per (D1D, Q1D): the H1 GLL basis at the
// Gauss-Legendre points is a pure function of the pair, so a table is written once per
// device (kern::upload_basis) and never changes.  The line kernel reads them through
// a pointer laundered at every stage (asm barrier), so the compiler issues scalar loads
// where they are used instead of hoisting 2*D*Q doubles out of the element loop (which
// exceeds the SGPR file and spills to VGPR lanes).
__constant__ Basis1D c_basis[MAX_D1D][MAX_Q1D];
typedef const __attribute__((address_space(4))) Basis1D CBasis;

template <int D, int Q>
__device__ __forceinline__ CBasis *stage_basis()
{
   CBasis *p = (CBasis *)&c_basis[D - 1][Q - 1];
   asm volatile("" : "+s"(p));
   return p;
}

template <int D, int Q, bool MASS, bool DIFF, bool AFF = false>
__device__ __forceinline__ void line_load_qdata(double (&qv)[7][Q], int e, int t,
                                                const double *__restrict__ qdd,
                                                const double *__restrict__ qdm)
{
   constexpr int NQ = Q * Q * Q, QQ = Q * Q;
   if (AFF && t < QQ)
   {
      // AFFINE_E: D_c = (W beta)(q) C_c, mass = (W alpha det J)(q); 16-byte pair per point
      double c[6];
#pragma unroll
      for (int k = 0; k < 6; k++) { c[k] = qdd[(size_t)e * 6 + k]; }
#pragma unroll
      for (int qz = 0; qz < Q; qz++)
      {
         const v2d p = reinterpret_cast<const v2d *>(qdm)[(size_t)e * NQ + qz * QQ + t];
#pragma unroll
         for (int k = 0; k < 6; k++) { qv[k][qz] = p.x * c[k]; }
         qv[6][qz] = p.y;
      }
      return;
   }
   if (t < QQ)
   {
#pragma unroll
      for (int qz = 0; qz < Q; qz++)
      {
         if (DIFF)
         {
#pragma unroll
            for (int c = 0; c < 6; c++) { qv[c][qz] = qdd[((size_t)e * 6 + c) * NQ + qz * QQ + t]; }
         }
         if (MASS) { qv[6][qz] = qdm[(size_t)e * NQ + qz * QQ + t]; }
      }
   }
}

// PA diagonal, one 64-lane workgroup per element, any qdata layout, any (D1D, Q1D) with
// Q1D^2 <= 64: the same seven terms sum-factorised in three stages through LDS --
// lanes (qx, qy) contract qz, lanes (qx, dz) contract qy, lanes (dy, dz) contract qx and
// add into the L-vector (atomics) or the E-vector.
template <int D, int Q>
__global__ void __launch_bounds__(64)
k_diag_sf(const int *__restrict__ pos, int kind, int ne, const int *__restrict__ gmap,
          const double *__restrict__ qdd, const double *__restrict__ qdm, double *__restrict__ diag, bool out_e)
{
   constexpr int ND = D * D * D, NQ = Q * Q * Q, QQ = Q * Q, DD = D * D, DQ = D * Q;
   static_assert(QQ <= 64, "k_diag_sf needs Q1D <= 8");
   __shared__ double T[7][D][QQ];   // [k][dz][qy qx]
   __shared__ double U[7][DD][Q];   // [k][dz dy][qx]
   const int e = blockIdx.x, t = threadIdx.x;
   if (e >= ne) { return; }
   CBasis *bp = stage_basis<D, Q>();
   // term k = fx(qx,dx) fy(qy,dy) fz(qz,dz) O_k: kinds 0 = B^2, 1 = G^2, 2 = G B per direction
   constexpr int FX[7] = {1, 0, 0, 2, 2, 0, 0}, FY[7] = {0, 1, 0, 2, 0, 2, 0}, FZ[7] = {0, 0, 1, 0, 2, 2, 0};
   auto f = [&](int kindf, int qq, int dd) {
      const double bq = bp->B[qq + MQ * dd], gq = bp->G[qq + MQ * dd];
      return kindf == 0 ? bq * bq : (kindf == 1 ? gq * gq : gq * bq);
   };
   if (t < QQ)
   {
      double acc[7][D];
#pragma unroll
      for (int k = 0; k < 7; k++)
#pragma unroll
         for (int dz = 0; dz < D; dz++) { acc[k][dz] = 0.0; }
#pragma unroll
      for (int qz = 0; qz < Q; qz++)
      {
         const int q = qz * QQ + t;
         double O[7];
         // symmetric entries (11,12,13,22,23,33) -> terms (11, 22, 33, 2*12, 2*13, 2*23), mass
         const int src[6] = {0, 3, 5, 1, 2, 4};
#pragma unroll
         for (int k = 0; k < 6; k++)
         {
            O[k] = qdd ? qd_diff_at(qdd, qdm, pos, kind, NQ, e, src[k], q) * (k >= 3 ? 2.0 : 1.0) : 0.0;
         }
         O[6] = qdm ? qd_mass_at(qdm, pos, kind, NQ, e, q) : 0.0;
#pragma unroll
         for (int k = 0; k < 7; k++)
#pragma unroll
            for (int dz = 0; dz < D; dz++) { acc[k][dz] += f(FZ[k], qz, dz) * O[k]; }
      }
#pragma unroll
      for (int k = 0; k < 7; k++)
#pragma unroll
         for (int dz = 0; dz < D; dz++) { T[k][dz][t] = acc[k][dz]; }
   }
   __syncthreads();
   if (t < DQ)
   {
      const int qx = t % Q, dz = t / Q;
#pragma unroll
      for (int k = 0; k < 7; k++)
#pragma unroll
         for (int dy = 0; dy < D; dy++)
         {
            double u = 0.0;
#pragma unroll
            for (int qy = 0; qy < Q; qy++) { u += f(FY[k], qy, dy) * T[k][dz][qy * Q + qx]; }
            U[k][dz * D + dy][qx] = u;
         }
   }
   __syncthreads();
   if (t < DD)
   {
#pragma unroll
      for (int dx = 0; dx < D; dx++)
      {
         double v = 0.0;
#pragma unroll
         for (int k = 0; k < 7; k++)
#pragma unroll
            for (int qx = 0; qx < Q; qx++) { v += f(FX[k], qx, dx) * U[k][t][qx]; }
         const long i = (long)e * ND + t * D + dx;
         if (out_e) { diag[i] += v; }
         else { unsafeAtomicAdd(diag + dof_of(gmap[i]), v); }
      }
   }
}

// As line_load_qdata with 16-byte loads from the native layout (even Q1D, lane pairs of
// adjacent columns l0 = l & ~1): lane l0 loads plane 2j and lane l0+1 plane 2j+1 of the
// pair's two columns, then each swaps the value its partner owns with one quad_perm DPP
// move -- half the load instructions, whole 16-byte segments per lane.
__device__ __forceinline__ double dpp_swap_pair(double v)
{
   const int lo = __double2loint(v), hi = __double2hiint(v);
   const int slo = __builtin_amdgcn_mov_dpp(lo, 0xB1, 0xF, 0xF, false);  // quad_perm(1,0,3,2)
   const int shi = __builtin_amdgcn_mov_dpp(hi, 0xB1, 0xF, 0xF, false);
   return __hiloint2double(shi, slo);
}

template <int D, int Q, bool MASS, bool DIFF>
__device__ __forceinline__ void line_load_qdata_x2(double (&qv)[7][Q], int e, int l,
                                                   const double *__restrict__ qdd,
                                                   const double *__restrict__ qdm)
{
   static_assert(Q % 2 == 0, "paired qdata loads need an even Q1D");
   constexpr int NQ = Q * Q * Q, QQ = Q * Q;
   const int odd = l & 1, l0 = l & ~1;
   auto pair = [&](const double *p, double &lo_plane, double &hi_plane) {
      const v2d v = *reinterpret_cast<const v2d *>(p);
      const double recv = dpp_swap_pair(odd ? v.x : v.y);
      lo_plane = odd ? recv : v.x;   // plane 2j of column l
      hi_plane = odd ? v.y : recv;   // plane 2j+1 of column l
   };
#pragma unroll
   for (int j = 0; j < Q / 2; j++)
   {
      const int qz = 2 * j + odd;
      if (DIFF)
      {
#pragma unroll
         for (int c = 0; c < 6; c++) { pair(qdd + ((size_t)e * 6 + c) * NQ + qz * QQ + l0, qv[c][2 * j], qv[c][2 * j + 1]); }
      }
      if (MASS) { pair(qdm + (size_t)e * NQ + qz * QQ + l0, qv[6][2 * j], qv[6][2 * j + 1]); }
   }
}

// Grid-function coefficient at the quadrature points (GridFunctionCoefficient projected
// by CoefficientVector::Project, coefficient.cpp:2052-2070 / qfunction.cpp:73-98, composed
// with the affine Pennes law), sum-factorised like the line kernel: one wave per element,
// lanes (dy,dz) gather a T x-line and contract in x, lanes (qx,dz) in y, lanes (qx,qy) in z;
// out[e][q] (q = qx + Q(qy + Q qz)) = scale * (1 + slope * (T(x_q) - t_ref)).
template <int D, int Q>
__global__ void __launch_bounds__(64)
k_coeff_line(int ne, const int *__restrict__ gmap, const double *__restrict__ T, double scale, double slope,
             double t_ref, double *__restrict__ out)
{
   constexpr int ND = D * D * D, NQ = Q * Q * Q, DD = D * D, QQ = Q * Q, DQ = D * Q;
   __shared__ double s1[DD * Q];
   __shared__ double s2[D * QQ];
   const int e = blockIdx.x, t = threadIdx.x;
   if (e >= ne) { return; }
   if (t < DD)
   {
      CBasis *bp = stage_basis<D, Q>();
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
      CBasis *bp = stage_basis<D, Q>();
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
      CBasis *bp = stage_basis<D, Q>();
      double l[D];
#pragma unroll
      for (int dz = 0; dz < D; dz++) { l[dz] = s2[dz * QQ + t]; }
#pragma unroll
      for (int qz = 0; qz < Q; qz++)
      {
         double v = 0.0;
#pragma unroll
         for (int dz = 0; dz < D; dz++) { v += bp->B[qz + MQ * dz] * l[dz]; }
         out[(size_t)e * NQ + qz * QQ + t] = scale * (1.0 + slope * (v - t_ref));
      }
   }
}

template <int D, int Q, bool MASS, bool DIFF, bool SPLIT, int VAR>
__global__ void __launch_bounds__(64)
k_apply_line(int c_begin, int c_end, const int *__restrict__ chunks, int n_owned,
             const int *__restrict__ gmap,
             const double *__restrict__ qdd, const double *__restrict__ qdm,
             const double *__restrict__ x, const double *__restrict__ xg,
             double *__restrict__ y, double *__restrict__ yg, const Basis1D b,
             double *__restrict__ part)
{
   constexpr int ND = D * D * D, DD = D * D, QQ = Q * Q, DQ = D * Q;
   constexpr int SA = (2 * DD * Q > 3 * D * QQ) ? 2 * DD * Q : 3 * D * QQ;
   constexpr int SB = (3 * D * QQ > 2 * DD * Q) ? 3 * D * QQ : 2 * DD * Q;
   static_assert(QQ <= 64, "line kernel needs Q1D <= 8");
   __shared__ double bufA[SA];  // s1, then s3
   __shared__ double bufB[SB];  // s2, then s4
   const int c = c_begin + ((VAR & 4) ? xcd_contiguous(blockIdx.x, gridDim.x) : (int)blockIdx.x);
   if (c >= c_end) { return; }  // whole wave
   const int t = threadIdx.x;
   const int ch = chunks[c];
   const int e0 = ch & 0xffffff, cnt = (VAR & 8) ? 1 : (ch >> 24);  // VAR & 8: one element per wave

   double qv[7][Q];
   if (!(VAR & 34)) { line_load_qdata<D, Q, MASS, DIFF, (VAR & 64) != 0>(qv, e0, t, qdd, qdm); }
   double carry = 0.0;
#pragma unroll 1
   for (int k = 0; k < cnt; k++)
   {
      const int e = e0 + k;
      if ((VAR & 2) && !(VAR & 32)) { line_load_qdata<D, Q, MASS, DIFF, (VAR & 64) != 0>(qv, e, t, qdd, qdm); }
      // ---- lanes (dy, dz): gather the x-line, contract in x
      int gl[D];
      if (t < DD)
      {
         CBasis *bp = stage_basis<D, Q>();
         const int *mp = gmap + (size_t)e * ND + t * D;
         double xl[D];
#pragma unroll
         for (int dx = 0; dx < D; dx++)
         {
            const int g = mp[dx];
            gl[dx] = g;
            const int d = bdof(g);
            const double v = (!SPLIT || d < n_owned) ? x[d] : xg[d - n_owned];
            xl[dx] = bneg(g) ? -v : v;
         }
#pragma unroll
         for (int qx = 0; qx < Q; qx++)
         {
            double u = 0.0, v = 0.0;
#pragma unroll
            for (int dx = 0; dx < D; dx++)
            {
               u += bp->B[qx + MQ * dx] * xl[dx];
               v += bp->G[qx + MQ * dx] * xl[dx];
            }
            bufA[t * Q + qx] = u;            // B_x   [dz][dy][qx]
            bufA[DD * Q + t * Q + qx] = v;   // G_x
         }
      }
      __syncthreads();
      // ---- lanes (qx, dz): contract in y
      if (t < DQ)
      {
         CBasis *bp = stage_basis<D, Q>();
         const int qx = t % Q, dz = t / Q;
         double la[D], lb[D];
#pragma unroll
         for (int dy = 0; dy < D; dy++)
         {
            la[dy] = bufA[(dz * D + dy) * Q + qx];
            lb[dy] = bufA[DD * Q + (dz * D + dy) * Q + qx];
         }
#pragma unroll
         for (int qy = 0; qy < Q; qy++)
         {
            double gb = 0.0, bg = 0.0, bb = 0.0;
#pragma unroll
            for (int dy = 0; dy < D; dy++)
            {
               const double by = bp->B[qy + MQ * dy], gy = bp->G[qy + MQ * dy];
               gb += by * lb[dy];  // G_x B_y
               bg += gy * la[dy];  // B_x G_y
               bb += by * la[dy];  // B_x B_y
            }
            const int o = (dz * Q + qy) * Q + qx;
            bufB[o] = gb;
            bufB[D * QQ + o] = bg;
            bufB[2 * D * QQ + o] = bb;
         }
      }
      __syncthreads();
      // ---- lanes (qx, qy): contract in z, weight at the quadrature points, transpose in z
      if (t < QQ)
      {
         CBasis *bp = stage_basis<D, Q>();
         double l0[D], l1[D], l2[D];
#pragma unroll
         for (int dz = 0; dz < D; dz++)
         {
            l0[dz] = bufB[dz * QQ + t];
            l1[dz] = bufB[D * QQ + dz * QQ + t];
            l2[dz] = bufB[2 * D * QQ + dz * QQ + t];
         }
         double A1[D], A2[D], A3[D];
#pragma unroll
         for (int dz = 0; dz < D; dz++) { A1[dz] = 0.0; A2[dz] = 0.0; A3[dz] = 0.0; }
         if (VAR & 32) { line_load_qdata<D, Q, MASS, DIFF, (VAR & 64) != 0>(qv, e, t, qdd, qdm); }  // just in time
#pragma unroll
         for (int qz = 0; qz < Q; qz++)
         {
            double gx = 0.0, gy = 0.0, gz = 0.0, u = 0.0;
#pragma unroll
            for (int dz = 0; dz < D; dz++)
            {
               const double bz = bp->B[qz + MQ * dz], gzz = bp->G[qz + MQ * dz];
               if (DIFF)
               {
                  gx += bz * l0[dz];
                  gy += bz * l1[dz];
                  gz += gzz * l2[dz];
               }
               if (MASS) { u += bz * l2[dz]; }
            }
            double fx = 0.0, fy = 0.0, fz = 0.0, m = 0.0;
            if (DIFF)
            {
               fx = qv[0][qz] * gx + qv[1][qz] * gy + qv[2][qz] * gz;
               fy = qv[1][qz] * gx + qv[3][qz] * gy + qv[4][qz] * gz;
               fz = qv[2][qz] * gx + qv[4][qz] * gy + qv[5][qz] * gz;
            }
            if (MASS) { m = qv[6][qz] * u; }
#pragma unroll
            for (int dz = 0; dz < D; dz++)
            {
               const double bz = bp->B[qz + MQ * dz], gzz = bp->G[qz + MQ * dz];
               if (DIFF)
               {
                  A1[dz] += bz * fx;               // -> G_x B_y
                  A2[dz] += bz * fy;               // -> B_x G_y
                  A3[dz] += gzz * fz;              // -> B_x B_y
               }
               if (MASS) { A3[dz] += bz * m; }    // -> B_x B_y
            }
         }
#pragma unroll
         for (int dz = 0; dz < D; dz++)
         {
            bufA[dz * QQ + t] = A1[dz];
            bufA[D * QQ + dz * QQ + t] = A2[dz];
            bufA[2 * D * QQ + dz * QQ + t] = A3[dz];
         }
      }
      // next element's qdata: in flight during the rest of this element
      if (!(VAR & 34) && k + 1 < cnt) { line_load_qdata<D, Q, MASS, DIFF, (VAR & 64) != 0>(qv, e + 1, t, qdd, qdm); }
      __syncthreads();
      // ---- lanes (qx, dz): transpose in y
      if (t < DQ)
      {
         CBasis *bp = stage_basis<D, Q>();
         const int qx = t % Q, dz = t / Q;
         double l0[Q], l1[Q], l2[Q];
#pragma unroll
         for (int qy = 0; qy < Q; qy++)
         {
            const int o = (dz * Q + qy) * Q + qx;
            l0[qy] = bufA[o];
            l1[qy] = bufA[D * QQ + o];
            l2[qy] = bufA[2 * D * QQ + o];
         }
#pragma unroll
         for (int dy = 0; dy < D; dy++)
         {
            double c1 = 0.0, c2 = 0.0;
#pragma unroll
            for (int qy = 0; qy < Q; qy++)
            {
               const double by = bp->B[qy + MQ * dy], gy = bp->G[qy + MQ * dy];
               c1 += by * l0[qy];                 // -> G_x
               c2 += gy * l1[qy] + by * l2[qy];   // -> B_x
            }
            bufB[(dz * D + dy) * Q + qx] = c1;
            bufB[DD * Q + (dz * D + dy) * Q + qx] = c2;
         }
      }
      __syncthreads();
      // ---- lanes (dy, dz): transpose in x, face carry, scatter
      if (t < DD)
      {
         CBasis *bp = stage_basis<D, Q>();
         double l0[Q], l1[Q];
#pragma unroll
         for (int qx = 0; qx < Q; qx++)
         {
            l0[qx] = bufB[t * Q + qx];
            l1[qx] = bufB[DD * Q + t * Q + qx];
         }
         const bool last = (k + 1 == cnt);
#pragma unroll
         for (int dx = 0; dx < D; dx++)
         {
            double v = 0.0;
#pragma unroll
            for (int qx = 0; qx < Q; qx++) { v += bp->G[qx + MQ * dx] * l0[qx] + bp->B[qx + MQ * dx] * l1[qx]; }
            const int g = gl[dx];
            if (bneg(g)) { v = -v; }
            if (dx == 0) { v += carry; }
            if (dx == D - 1 && !last)
            {
               carry = v;  // summed into the next element's (0, dy, dz) entry
               continue;
            }
            const int d = bdof(g);
            double *dst = (!SPLIT || d < n_owned) ? y + d : yg + (d - n_owned);
            if (!bshared(g)) { *dst = v; }
            else if (part) { part[(size_t)e * ND + t * D + dx] = v; }
            else { unsafeAtomicAdd(dst, v); }
         }
      }
      // no barrier here: the next element writes bufA (last read before barrier 4) and,
      // after its first barrier, bufB (last read above)
   }
}

// --------------------------------------------------------------------------
// Brick kernel (p >= 3): one workgroup per brick of 2 x 2 x BZ elements whose internal
// faces coincide (found by dof equality at setup, pa_form.cpp).  The five 1D stages of
// the line kernel run for all elements of the brick at once, lane = (element, line), so
// the 25 / 30 / 36-line stages of a p = 4 element fill 4-5 waves instead of leaving half
// of one wave idle.  The elements' outputs are then summed on the brick lattice
// ((2(D-1)+1)^2 (BZ(D-1)+1) points) in LDS in a fixed order, so the shared faces inside
// a brick never reach HBM: a lattice point held by this brick alone is plain-stored,
// one on the brick surface that other holders share goes to its partial slot
// part[brick][surface index] (face-grouped, brick_surface_index) for k_sum_partials
// (deterministic, no atomics).
// Per element: same qdata, x-line gathers and contractions as k_apply_line
// (bilininteg_mass_kernels.hpp:809-1033, bilininteg_diffusion_kernels.hpp:989-1214);
// the brick map replaces ElementRestriction's element maps (restriction.cpp:109-186).
// --------------------------------------------------------------------------
template <int D, int Q, int BZ>
struct BrickShape
{
   // BZ <= 2: all 4 BZ elements at once; BZ > 2 (column bricks): NL = BZ layers of 2 x 2
   // elements marched in z by one workgroup, each layer's top lattice plane carried in LDS
   // into the next layer's bottom plane, so the column's internal z faces never reach HBM
   static constexpr int NL = BZ > 2 ? BZ : 1, NET = 4 * BZ;
   static constexpr int NE = 4 * (BZ > 2 ? 1 : BZ), DD = D * D, QQ = Q * Q, DQ = D * Q, ND = D * D * D;
   static constexpr int LX = 2 * (D - 1) + 1, LY = LX, LZ = BZ * (D - 1) + 1, NB = LX * LY * LZ;
   static constexpr int NBL = LX * LY * ((BZ > 2 ? 1 : BZ) * (D - 1) + 1);  // lattice points per pass
   static constexpr int SURF = 2 * LX * LY + 2 * (LZ - 2) * LX + 2 * (LZ - 2) * (LY - 2);
   // per-element LDS: SA holds the x-stage lines (2 D^2 Q), SB the y/z-stage planes (3 D Q^2,
   // the z stage works in place); staged element outputs (D^3) reuse SB
   static constexpr int SA = 2 * DD * Q, SB = 3 * D * QQ;
   static constexpr int NT = ((NE * QQ + 63) / 64) * 64;  // stage 3 in one pass
   // waves per SIMD the register budget targets: 4 (<= 128 VGPRs) up to p = 4, where the
   // 2 x 2 x 1 brick then fits 5 workgroups per CU; the larger orders keep their registers
   static constexpr int WPE = D <= 5 ? 4 : 1;
};

// lattice coordinate P along one brick direction -> (first element index, local index,
// holders): the shared plane P = D-1 is held by element 0 (local D-1) and 1 (local 0)
template <int D>
__device__ __forceinline__ void brick_cand(int P, int &c0, int &l0, int &n)
{
   if (P < D - 1) { c0 = 0; l0 = P; n = 1; }
   else if (P == D - 1) { c0 = 0; l0 = D - 1; n = 2; }
   else { c0 = 1; l0 = P - (D - 1); n = 1; }
}

// (ECM2_BRICK_VARIANT bit 8 selects VAR bit 256, the XCD-contiguous order, on AFFINE_E.)
// VAR bit 1: load the stage-3 qdata at the top of the z stage (fewer VGPRs, more
// workgroups per CU) instead of at kernel entry (in flight during stages 1-2); bit 2:
// 16-byte paired loads (line_load_qdata_x2, even Q1D); bit 128: one LDS buffer of
// 3 D Q^2 doubles per element instead of two (2 D^2 Q + 3 D Q^2): each stage reads its
// lines into registers, waits at a barrier, then overwrites the buffer (three more
// barriers, 36% less LDS: 9 instead of 5 p = 4 workgroups per CU)
template <int D, int Q, int BZ, bool MASS, bool DIFF, bool SPLIT, int VAR>
__global__ void __launch_bounds__((BrickShape<D, Q, BZ>::NT),
                                  ((VAR & 128) && D <= 5 ? 5 : BrickShape<D, Q, BZ>::WPE))
k_apply_brick(int k_begin, int k_end, const int *__restrict__ belem, const int *__restrict__ bmap, int n_owned,
              const double *__restrict__ qdd, const double *__restrict__ qdm,
              const double *__restrict__ x, const double *__restrict__ xg,
              double *__restrict__ y, double *__restrict__ yg, double *__restrict__ part)
{
   using S = BrickShape<D, Q, BZ>;
   constexpr int NE = S::NE, DD = S::DD, QQ = S::QQ, DQ = S::DQ, ND = S::ND, SA = S::SA, SB = S::SB;
   constexpr int LX = S::LX, LY = S::LY, NB = S::NB;
   static_assert(QQ <= 64, "brick kernel needs Q1D <= 8");
   static_assert(SB >= ND, "staged outputs reuse bufB");
   constexpr bool ONE = (VAR & 128) != 0;
   static_assert(SB >= SA, "one-buffer variant");
   __shared__ double bufA[ONE ? 1 : NE * SA];
   __shared__ double bufB[NE * SB];
   double *const sA = ONE ? bufB : bufA;  // the x-stage lines
   // VAR bit 256: XCD-contiguous brick order (neighbouring bricks share x values and
   // partial-slot lines: keep them in one XCD's L2)
   const int k = k_begin + ((VAR & 256) ? xcd_contiguous(blockIdx.x, gridDim.x) : (int)blockIdx.x);
   if (k >= k_end) { return; }  // whole workgroup
   const int t = threadIdx.x;
   const int *bm = bmap + (size_t)k * NB;
   auto lattice = [&](int elt, int dx, int dy, int dz) {
      const int ex = elt & 1, ey = (elt >> 1) & 1, ez = elt >> 2;
      return ((ez * (D - 1) + dz) * LY + ey * (D - 1) + dy) * LX + ex * (D - 1) + dx;
   };

   __shared__ double carry[S::NL > 1 ? 2 * LX * LY : 1];  // column bricks: top plane -> next layer
#pragma unroll
   for (int layer = 0; layer < S::NL; layer++)
   {
   const int eo = layer * NE;  // this pass's first element in the brick
   const int *be = belem + (size_t)k * S::NET + eo;
   // qdata of the (element, qx, qy) column this lane weights in stage 3: in flight
   // during the gather and the x / y contractions
   double qv[7][Q];
   // AFFINE_E (VAR & 64): the raw per-point pairs and the element's C stay in registers until
   // the z stage (forming the 6 entries at load time would make the wave wait for the loads
   // at entry, and hold 7Q values instead of 2Q + 6)
   constexpr bool AFF = (VAR & 64) != 0;
   v2d pa[Q];
   double cc[6];
   if (AFF && !(VAR & 1) && t < NE * QQ)
   {
      const int e = be[t / QQ], l = t % QQ;
      constexpr int NQ = Q * Q * Q;
#pragma unroll
      for (int qz = 0; qz < Q; qz++) { pa[qz] = reinterpret_cast<const v2d *>(qdm)[(size_t)e * NQ + qz * QQ + l]; }
#pragma unroll
      for (int c = 0; c < 6; c++) { cc[c] = qdd[(size_t)e * 6 + c]; }
   }
   if (!AFF && !(VAR & 1) && t < NE * QQ)
   {
      if constexpr ((VAR & 2) && Q % 2 == 0)
      {
         line_load_qdata_x2<D, Q, MASS, DIFF>(qv, be[t / QQ], t % QQ, qdd, qdm);
      }
      else { line_load_qdata<D, Q, MASS, DIFF, (VAR & 64) != 0>(qv, be[t / QQ], t % QQ, qdd, qdm); }
   }

   // ---- lanes (element, dy, dz): gather the x-line, contract in x
   if (t < NE * DD)
   {
      CBasis *bp = stage_basis<D, Q>();
      const int elt = t / DD, l = t % DD;
      const int *mp = bm + lattice(eo + elt, 0, l % D, l / D);
      double xl[D];
#pragma unroll
      for (int dx = 0; dx < D; dx++)
      {
         const int d = bdof(mp[dx]);
         xl[dx] = (!SPLIT || d < n_owned) ? x[d] : xg[d - n_owned];
      }
      double *o = sA + elt * (ONE ? SB : SA);
#pragma unroll
      for (int qx = 0; qx < Q; qx++)
      {
         double u = 0.0, v = 0.0;
#pragma unroll
         for (int dx = 0; dx < D; dx++)
         {
            u += bp->B[qx + MQ * dx] * xl[dx];
            v += bp->G[qx + MQ * dx] * xl[dx];
         }
         o[l * Q + qx] = u;
         o[DD * Q + l * Q + qx] = v;
      }
   }
   __syncthreads();
   // ---- lanes (element, qx, dz): contract in y
   double la[D], lb[D];
   if (t < NE * DQ)
   {
      const int elt = t / DQ, l = t % DQ, qx = l % Q, dz = l / Q;
      const double *in = sA + elt * (ONE ? SB : SA);
#pragma unroll
      for (int dy = 0; dy < D; dy++)
      {
         la[dy] = in[(dz * D + dy) * Q + qx];
         lb[dy] = in[DD * Q + (dz * D + dy) * Q + qx];
      }
   }
   if (ONE) { __syncthreads(); }
   if (t < NE * DQ)
   {
      CBasis *bp = stage_basis<D, Q>();
      const int elt = t / DQ, l = t % DQ, qx = l % Q, dz = l / Q;
      double *o = bufB + elt * SB;
#pragma unroll
      for (int qy = 0; qy < Q; qy++)
      {
         double gb = 0.0, bg = 0.0, bb = 0.0;
#pragma unroll
         for (int dy = 0; dy < D; dy++)
         {
            const double by = bp->B[qy + MQ * dy], gy = bp->G[qy + MQ * dy];
            gb += by * lb[dy];
            bg += gy * la[dy];
            bb += by * la[dy];
         }
         const int oo = (dz * Q + qy) * Q + qx;
         o[oo] = gb;
         o[D * QQ + oo] = bg;
         o[2 * D * QQ + oo] = bb;
      }
   }
   __syncthreads();
   // ---- lanes (element, qx, qy): contract in z, weight, transpose in z (in place: a lane
   // reads its whole (qx, qy) column before writing it back)
   if (t < NE * QQ)
   {
      CBasis *bp = stage_basis<D, Q>();
      const int elt = t / QQ, l = t % QQ;
      if (!AFF && (VAR & 1)) { line_load_qdata<D, Q, MASS, DIFF, false>(qv, be[elt], l, qdd, qdm); }
      // AFFINE_E, VAR bit 1: C_e here, the per-point pairs inside the qz loop (fewer live VGPRs)
      const v2d *pz = reinterpret_cast<const v2d *>(qdm) + (size_t)be[elt] * (Q * QQ) + l;
      if (AFF && (VAR & 1))
      {
#pragma unroll
         for (int c = 0; c < 6; c++) { cc[c] = qdd[(size_t)be[elt] * 6 + c]; }
      }
      double *in = bufB + elt * SB;
      double *o = in;
      double l0[D], l1[D], l2[D];
#pragma unroll
      for (int dz = 0; dz < D; dz++)
      {
         l0[dz] = in[dz * QQ + l];
         l1[dz] = in[D * QQ + dz * QQ + l];
         l2[dz] = in[2 * D * QQ + dz * QQ + l];
      }
      double A1[D], A2[D], A3[D];
#pragma unroll
      for (int dz = 0; dz < D; dz++) { A1[dz] = 0.0; A2[dz] = 0.0; A3[dz] = 0.0; }
#pragma unroll
      for (int qz = 0; qz < Q; qz++)
      {
         double gx = 0.0, gy = 0.0, gz = 0.0, u = 0.0;
#pragma unroll
         for (int dz = 0; dz < D; dz++)
         {
            const double bz = bp->B[qz + MQ * dz], gzz = bp->G[qz + MQ * dz];
            if (DIFF)
            {
               gx += bz * l0[dz];
               gy += bz * l1[dz];
               gz += gzz * l2[dz];
            }
            if (MASS) { u += bz * l2[dz]; }
         }
         double fx = 0.0, fy = 0.0, fz = 0.0, m = 0.0;
         if (AFF && (VAR & 1)) { pa[qz] = pz[qz * QQ]; }
         if (DIFF)
         {
            if (AFF)
            {
               const double wb = pa[qz].x;
               fx = wb * (cc[0] * gx + cc[1] * gy + cc[2] * gz);
               fy = wb * (cc[1] * gx + cc[3] * gy + cc[4] * gz);
               fz = wb * (cc[2] * gx + cc[4] * gy + cc[5] * gz);
            }
            else
            {
               fx = qv[0][qz] * gx + qv[1][qz] * gy + qv[2][qz] * gz;
               fy = qv[1][qz] * gx + qv[3][qz] * gy + qv[4][qz] * gz;
               fz = qv[2][qz] * gx + qv[4][qz] * gy + qv[5][qz] * gz;
            }
         }
         if (MASS) { m = (AFF ? pa[qz].y : qv[6][qz]) * u; }
#pragma unroll
         for (int dz = 0; dz < D; dz++)
         {
            const double bz = bp->B[qz + MQ * dz], gzz = bp->G[qz + MQ * dz];
            if (DIFF)
            {
               A1[dz] += bz * fx;
               A2[dz] += bz * fy;
               A3[dz] += gzz * fz;
            }
            if (MASS) { A3[dz] += bz * m; }
         }
      }
#pragma unroll
      for (int dz = 0; dz < D; dz++)
      {
         o[dz * QQ + l] = A1[dz];
         o[D * QQ + dz * QQ + l] = A2[dz];
         o[2 * D * QQ + dz * QQ + l] = A3[dz];
      }
   }
   __syncthreads();
   // ---- lanes (element, qx, dz): transpose in y
   double t0[Q], t1[Q], t2[Q];
   if (t < NE * DQ)
   {
      const int elt = t / DQ, l = t % DQ, qx = l % Q, dz = l / Q;
      const double *in = bufB + elt * SB;
#pragma unroll
      for (int qy = 0; qy < Q; qy++)
      {
         const int oo = (dz * Q + qy) * Q + qx;
         t0[qy] = in[oo];
         t1[qy] = in[D * QQ + oo];
         t2[qy] = in[2 * D * QQ + oo];
      }
   }
   if (ONE) { __syncthreads(); }
   if (t < NE * DQ)
   {
      CBasis *bp = stage_basis<D, Q>();
      const int elt = t / DQ, l = t % DQ, qx = l % Q, dz = l / Q;
      double *o = sA + elt * (ONE ? SB : SA);
      const double *l0 = t0, *l1 = t1, *l2 = t2;
#pragma unroll
      for (int dy = 0; dy < D; dy++)
      {
         double c1 = 0.0, c2 = 0.0;
#pragma unroll
         for (int qy = 0; qy < Q; qy++)
         {
            const double by = bp->B[qy + MQ * dy], gy = bp->G[qy + MQ * dy];
            c1 += by * l0[qy];
            c2 += gy * l1[qy] + by * l2[qy];
         }
         o[(dz * D + dy) * Q + qx] = c1;
         o[DD * Q + (dz * D + dy) * Q + qx] = c2;
      }
   }
   __syncthreads();
   // ---- lanes (element, dy, dz): transpose in x -> element outputs staged in LDS [elt][a]
   double l0[Q], l1[Q];
   if (t < NE * DD)
   {
      const int elt = t / DD, l = t % DD;
      const double *in = sA + elt * (ONE ? SB : SA);
#pragma unroll
      for (int qx = 0; qx < Q; qx++)
      {
         l0[qx] = in[l * Q + qx];
         l1[qx] = in[DD * Q + l * Q + qx];
      }
   }
   if (ONE) { __syncthreads(); }
   if (t < NE * DD)
   {
      CBasis *bp = stage_basis<D, Q>();
      const int elt = t / DD, l = t % DD;
#pragma unroll
      for (int dx = 0; dx < D; dx++)
      {
         double v = 0.0;
#pragma unroll
         for (int qx = 0; qx < Q; qx++) { v += bp->G[qx + MQ * dx] * l0[qx] + bp->B[qx + MQ * dx] * l1[qx]; }
         bufB[elt * ND + l * D + dx] = v;  // bufB is free: stage 4 (ONE: stage 5) read it before a barrier
      }
   }
   __syncthreads();
   // ---- lattice points: sum the holders in a fixed (z, y, x) order, store or publish
   for (int p = t; p < S::NBL; p += S::NT)
   {
      const int X = p % LX, Y = (p / LX) % LY, Z = p / (LX * LY);  // Z within this pass
      int cx, lx, nx, cy, ly, ny, cz, lz, nz;
      brick_cand<D>(X, cx, lx, nx);
      brick_cand<D>(Y, cy, ly, ny);
      if (BZ == 2) { brick_cand<D>(Z, cz, lz, nz); }
      else { cz = 0; lz = Z; nz = 1; }
      double v = 0.0;
      for (int iz = 0; iz < nz; iz++)
         for (int iy = 0; iy < ny; iy++)
            for (int ix = 0; ix < nx; ix++)
            {
               const int elt = (cx + ix) + 2 * ((cy + iy) + 2 * (cz + iz));
               const int a = ((iz ? 0 : lz) * D + (iy ? 0 : ly)) * D + (ix ? 0 : lx);
               v += bufB[elt * ND + a];
            }
      if constexpr (S::NL > 1)
      {
         if (Z == 0 && layer > 0) { v += carry[((layer - 1) & 1) * LX * LY + Y * LX + X]; }
         if (Z == D - 1 && layer < S::NL - 1)
         {
            carry[(layer & 1) * LX * LY + Y * LX + X] = v;  // completed by the next layer
            continue;
         }
      }
      const int zg = layer * (D - 1) + Z;  // lattice plane in the whole brick
      const int g = bm[p + layer * (D - 1) * LX * LY];
      const int d = bdof(g);
      if (!bshared(g)) { *((!SPLIT || d < n_owned) ? y + d : yg + (d - n_owned)) = v; }
      else { part[(size_t)k * S::SURF + brick_surface_index(D, BZ, X, Y, zg)] = v; }  // surface only (setup)
   }
   // the next layer's first writes (bufA; ONE: bufB) follow reads of this pass's last
   // stages behind barriers, except in the one-buffer variant
   if (S::NL > 1 && ONE) { __syncthreads(); }
   }
}

__global__ void k_restriction_mult(long n, const int *__restrict__ gmap,
                                   const double *__restrict__ x, double *__restrict__ xe)
{
   const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
   if (i >= n) { return; }
   const int g = gmap[i];
   const double v = x[dof_of(g)];
   xe[i] = g >= 0 ? v : -v;
}

__global__ void k_restriction_mult_transpose(int ndofs, const int *__restrict__ offsets,
                                             const int *__restrict__ indices,
                                             const double *__restrict__ xe,
                                             double *__restrict__ y)
{
   const int i = blockIdx.x * blockDim.x + threadIdx.x;
   if (i >= ndofs) { return; }
   double v = 0.0;
   for (int j = offsets[i]; j < offsets[i + 1]; j++)
   {
      const int idx = indices[j];
      v += idx >= 0 ? xe[idx] : -xe[-1 - idx];
   }
   y[i] = v;
}

__global__ void k_diagonal(const int *__restrict__ pos, int D, int Q, int kind, int ne, const int *__restrict__ gmap,
                           const double *__restrict__ qdd, const double *__restrict__ qdm,
                           double *__restrict__ diag, bool out_e, const Basis1D b)
{
   const int ND = D * D * D, NQ = Q * Q * Q;
   const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
   if (t >= (long)ne * ND) { return; }
   const int e = (int)(t / ND), a = (int)(t % ND);
   const int dx = a % D, dy = (a / D) % D, dz = a / (D * D);
   double s = 0.0;
   for (int qz = 0; qz < Q; qz++)
      for (int qy = 0; qy < Q; qy++)
         for (int qx = 0; qx < Q; qx++)
         {
            const int q = (qz * Q + qy) * Q + qx;
            const double bx = b.B[qx + MQ * dx], by = b.B[qy + MQ * dy], bz = b.B[qz + MQ * dz];
            const double gx = b.G[qx + MQ * dx], gy = b.G[qy + MQ * dy], gz = b.G[qz + MQ * dz];
            if (qdm) { s += bx * bx * by * by * bz * bz * qd_mass_at(qdm, pos, kind, NQ, e, q); }
            if (qdd)
            {
               const double p0 = gx * by * bz, p1 = bx * gy * bz, p2 = bx * by * gz;
               s += p0 * p0 * qd_diff_at(qdd, qdm, pos, kind, NQ, e, 0, q) +
                    p1 * p1 * qd_diff_at(qdd, qdm, pos, kind, NQ, e, 3, q) +
                    p2 * p2 * qd_diff_at(qdd, qdm, pos, kind, NQ, e, 5, q) +
                    2.0 * (p0 * p1 * qd_diff_at(qdd, qdm, pos, kind, NQ, e, 1, q) +
                           p0 * p2 * qd_diff_at(qdd, qdm, pos, kind, NQ, e, 2, q) +
                           p1 * p2 * qd_diff_at(qdd, qdm, pos, kind, NQ, e, 4, q));
            }
         }
   if (out_e) { diag[t] += s; }
   else { unsafeAtomicAdd(diag + dof_of(gmap[t]), s); }
}

__global__ void k_set_values(int n, const int *__restrict__ idx, double val, double *__restrict__ y)
{
   const int i = blockIdx.x * blockDim.x + threadIdx.x;
   if (i < n) { y[idx[i]] = val; }
}

__global__ void k_copy_values(int n, const int *__restrict__ idx, const double *__restrict__ x,
                              double *__restrict__ y)
{
   const int i = blockIdx.x * blockDim.x + threadIdx.x;
   if (i < n) { y[idx[i]] = x[idx[i]]; }
}

constexpr int kDotBlocks = 1024;

__global__ void __launch_bounds__(256)
k_dot_partial(int n, const double *__restrict__ a, const double *__restrict__ b,
              double *__restrict__ partials)
{
   __shared__ double red[4];
   double s = 0.0;
   for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
   {
      s += a[i] * b[i];
   }
   for (int off = 32; off > 0; off >>= 1) { s += __shfl_down(s, off, 64); }
   if ((threadIdx.x & 63) == 0) { red[threadIdx.x >> 6] = s; }
   __syncthreads();
   if (threadIdx.x == 0) { partials[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]); }
}

__global__ void __launch_bounds__(256)
k_dot_final(int nparts, const double *__restrict__ partials, double *__restrict__ out, double *__restrict__ hout)
{
   __shared__ double red[4];
   double s = 0.0;
   for (int i = threadIdx.x; i < nparts; i += blockDim.x) { s += partials[i]; }
   for (int off = 32; off > 0; off >>= 1) { s += __shfl_down(s, off, 64); }
   if ((threadIdx.x & 63) == 0) { red[threadIdx.x >> 6] = s; }
   __syncthreads();
   if (threadIdx.x == 0)
   {
      const double v = (red[0] + red[1]) + (red[2] + red[3]);
      *out = v;
      if (hout) { *hout = v; }  // mapped pinned host mirror (the solver's stopping test)
   }
}

__global__ void k_pcg_update_xr(int n, const double *__restrict__ nom,
                                const double *__restrict__ den, const double *__restrict__ d,
                                const double *__restrict__ z, double *__restrict__ x,
                                double *__restrict__ r)
{
   const int i = blockIdx.x * blockDim.x + threadIdx.x;
   if (i >= n) { return; }
   const double alpha = *nom / *den;
   x[i] = x[i] + alpha * d[i];
   r[i] = r[i] + (-alpha) * z[i];
}

// One fused PCG update (CGSolver::Mult's add/Mult(prec)/Dot sequence, solvers.cpp:930-960):
// alpha = nom/den; x += alpha d; r -= alpha Ad; z = dinv .* r (jacobi) ; partial sums of r.z
// (or r.r) in the fixed grid-stride order of k_dot_partial, finished by k_dot_final.
// z holds A d on entry and the preconditioned residual on exit (jacobi only).
__global__ void __launch_bounds__(256)
k_pcg_step(int n, const double *__restrict__ nom, const double *__restrict__ den,
           const double *__restrict__ d, double *__restrict__ z, double *__restrict__ x,
           double *__restrict__ r, const double *__restrict__ dinv, double *__restrict__ partials)
{
   __shared__ double red[4];
   const double alpha = *nom / *den;
   double s = 0.0;
   for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
   {
      x[i] = x[i] + alpha * d[i];
      const double rn = r[i] + (-alpha) * z[i];
      r[i] = rn;
      if (dinv)
      {
         const double zn = dinv[i] * rn;
         z[i] = zn;
         s += rn * zn;
      }
      else { s += rn * rn; }
   }
   for (int off = 32; off > 0; off >>= 1) { s += __shfl_down(s, off, 64); }
   if ((threadIdx.x & 63) == 0) { red[threadIdx.x >> 6] = s; }
   __syncthreads();
   if (threadIdx.x == 0) { partials[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]); }
}

// ConstrainedOperator around a Mult without a vector copy: saved = v[ess], v[ess] = 0 ...
__global__ void k_ess_save_zero(int n, const int *__restrict__ idx, double *__restrict__ v,
                                double *__restrict__ saved)
{
   const int i = blockIdx.x * blockDim.x + threadIdx.x;
   if (i < n) { saved[i] = v[idx[i]]; v[idx[i]] = 0.0; }
}

// ... then v[ess] = y[ess] = saved (DIAG_ONE rows)
__global__ void k_ess_restore(int n, const int *__restrict__ idx, const double *__restrict__ saved,
                              double *__restrict__ v, double *__restrict__ y)
{
   const int i = blockIdx.x * blockDim.x + threadIdx.x;
   if (i < n) { v[idx[i]] = saved[i]; y[idx[i]] = saved[i]; }
}

__global__ void k_pcg_precond(int n, const double *__restrict__ dinv, const double *__restrict__ r,
                              double *__restrict__ z)
{
   const int i = blockIdx.x * blockDim.x + threadIdx.x;
   if (i < n) { z[i] = dinv ? dinv[i] * r[i] : r[i]; }
}

__global__ void k_pcg_update_d(int n, const double *__restrict__ betanom,
                               const double *__restrict__ nom, const double *__restrict__ z,
                               double *__restrict__ d)
{
   const int i = blockIdx.x * blockDim.x + threadIdx.x;
   if (i >= n) { return; }
   const double beta = *betanom / *nom;
   d[i] = z[i] + beta * d[i];
}

__global__ void k_scale(int n, double a, double *__restrict__ y)
{
   const int i = blockIdx.x * blockDim.x + threadIdx.x;
   if (i < n) { y[i] *= a; }
}

// out = x + c k  (out may alias x)
__global__ void k_add_scaled(int n, const double *x, double c, const double *__restrict__ k, double *out)
{
   const int i = blockIdx.x * blockDim.x + threadIdx.x;
   if (i < n) { out[i] = x[i] + c * k[i]; }
}

// STREAM copy (measurement only): 16-byte nontemporal loads and stores, grid-stride,
// the access shape of the guide's 6.29 TB/s float4-copy figure.
__global__ void k_stream_copy(long n2, const v2d *__restrict__ a, v2d *__restrict__ b)
{
   const long stride = (long)gridDim.x * blockDim.x;
   for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += stride)
   {
      __builtin_nontemporal_store(__builtin_nontemporal_load(a + i), b + i);
   }
}

__global__ void k_reciprocal(int n, const double *__restrict__ a, double *__restrict__ out)
{
   const int i = blockIdx.x * blockDim.x + threadIdx.x;
   if (i < n) { out[i] = 1.0 / a[i]; }
}

__global__ void k_gather_idx(int n, const int *__restrict__ idx, const double *__restrict__ x,
                             double *__restrict__ buf)
{
   const int i = blockIdx.x * blockDim.x + threadIdx.x;
   if (i < n) { buf[i] = x[idx[i]]; }
}

__global__ void k_scatter_add_idx(int n, const int *__restrict__ idx, const double *__restrict__ buf,
                                  double *__restrict__ y)
{
   const int i = blockIdx.x * blockDim.x + threadIdx.x;
   // atomic: a dof shared by >= 3 ranks appears in several neighbour segments
   if (i < n) { unsafeAtomicAdd(y + idx[i], buf[i]); }
}

__global__ void k_scatter_set_idx(int n, const int *__restrict__ idx, const double *__restrict__ buf,
                                  double *__restrict__ y)
{
   const int i = blockIdx.x * blockDim.x + threadIdx.x;
   if (i < n) { y[idx[i]] = buf[i]; }
}

// Second pass of the deterministic scatter: y[dofs[i]] = sum of the partial slots
// slots[start .. start+count) in ascending slot order, for i in [i0, i1), with
// meta[i] = start << 5 | count.  All slot loads, then all partial loads, are issued
// independently (count <= 8 unrolled; more -- unstructured meshes -- loops), so a
// thread waits ~3 memory latencies instead of 2 + 2*count.  The list is ordered by
// first slot (pa_form.cpp), so neighbouring threads read neighbouring lanes.
// XCD: block b takes a contiguous range of blocks per XCD (xcd_contiguous), so the slot
// lines neighbouring dofs read sit in one L2
template <bool XCD>
__global__ void k_sum_partials(int i0, int i1, const int *__restrict__ dofs, const unsigned *__restrict__ meta,
                               const int *__restrict__ slots, const double *__restrict__ part, int n_owned,
                               double *__restrict__ y, double *__restrict__ yg)
{
   const int b = XCD ? xcd_contiguous(blockIdx.x, gridDim.x) : (int)blockIdx.x;
   const int i = i0 + b * blockDim.x + threadIdx.x;
   if (i >= i1) { return; }
   const unsigned m = meta[i];
   const int d = dofs[i];
   const int start = (int)(m >> 5), cnt = (int)(m & 31);
   double acc = 0.0;
   if (!slots)
   {
      // contiguous runs (pslot plan): the dof's holders are part[start, start + cnt)
      double v[8];
#pragma unroll
      for (int k = 0; k < 8; k++) { v[k] = k < cnt ? part[start + k] : 0.0; }
#pragma unroll
      for (int k = 0; k < 8; k++) { acc += v[k]; }
      for (int k = 8; k < cnt; k++) { acc += part[start + k]; }
   }
   else
   {
   int sl[8];
#pragma unroll
   for (int k = 0; k < 8; k++) { sl[k] = k < cnt ? slots[start + k] : -1; }
   double v[8];
#pragma unroll
   for (int k = 0; k < 8; k++) { v[k] = sl[k] >= 0 ? part[sl[k]] : 0.0; }
#pragma unroll
   for (int k = 0; k < 8; k++) { acc += v[k]; }
   for (int k = 8; k < cnt; k++) { acc += part[slots[start + k]]; }
   }
   if (d < n_owned) { y[d] = acc; }
   else { yg[d - n_owned] = acc; }
}

inline unsigned grid_for(long n, int bs) { return (unsigned)((n + bs - 1) / bs); }

SetupCoef make_setup_coef(const CoeffDesc *c, const double *q)
{
   SetupCoef s{};
   if (!c) { return s; }
   s.has = 1;
   s.is_const = (c->kind == COEFF_CONSTANT);
   s.value = c->value;
   s.quad = q;
   return s;
}

int tpe_variant()
{
   static int v = [] {
      const char *e = std::getenv("ECM2_TPE_VARIANT");
      return e ? std::atoi(e) : kDefaultTpeVariant;
   }();
   return v;
}

template <int D, int Q, bool MASS, bool DIFF, bool SPLIT>
void launch_tpe_pf(int var, const ApplyArgs &a, const Basis1D &b, const double *rowtab, hipStream_t s)
{
   const int nb = a.blk_end - a.blk_begin;
   const dim3 grid((nb + 3) / 4), block(256);
#define ECM2_PF_AF(V, AF)                                                                            \
   hipLaunchKernelGGL((k_apply_tpe_pf<D, Q, MASS, DIFF, SPLIT, V, AF>), grid, block, 0, s, a.ne,    \
                      a.blk_begin, a.blk_end, a.n_owned, a.gmap, a.qdd, a.qdm, a.x, a.xg, a.y, a.yg, b, rowtab, \
                      a.lane_flags, a.part, a.pslot)
#define ECM2_PF(V) ECM2_PF_AF(V, false)
   if (a.kind == QLAYOUT_AFFINE)
   {
      if constexpr (MASS && DIFF)
      {
         // experiment knob bits: 64 = the row kernel (k_apply_tpe_pf) instead of the plane-
         // factorised one, 2 = cached qdata loads, 8 = two waves per SIMD, 16 = XCD order
#define ECM2_SF(V)                                                                                   \
   hipLaunchKernelGGL((k_apply_tpe_sf<D, Q, SPLIT, V>), ((V) & 128) ? dim3((nb + 7) / 8) : grid,       \
                      ((V) & 128) ? dim3(512) : block, 0, s, a.ne, a.blk_begin, a.blk_end,            \
                      a.n_owned, a.gmap, a.qdd, a.qdm, a.x, a.xg, a.y, a.yg, b, a.lane_flags, a.part, a.pslot)
         if (a.latency)
         {
            hipLaunchKernelGGL((k_apply_tpe_pp<D, Q, SPLIT>), dim3(nb), dim3(256), 0, s, a.ne, a.blk_begin,
                               a.n_owned, a.gmap, a.qdd, a.qdm, a.x, a.xg, a.y, a.yg, b, a.lane_flags, a.part,
                               a.pslot);
         }
         else if (var & 64)
         {
            switch (var & 26)
            {
               case 2: ECM2_PF_AF(2, true); break;
               case 8: ECM2_PF_AF(8, true); break;
               case 16: ECM2_PF_AF(16, true); break;
               default: ECM2_PF_AF(0, true); break;
            }
         }
         else
         {
            if (a.xwg == 8) { ECM2_SF(128); }
            else
            switch (var & 14)
            {
               case 2: ECM2_SF(2); break;
               case 8: ECM2_SF(8); break;
               case 12: ECM2_SF(12); break;
               default:
                  if (var & 256) { ECM2_SF(4); }  // deep prefetch (bit 256 of the knob)
                  else if (var & 512) { ECM2_SF(32); }  // plane prefetch (bit 512)
                  else { ECM2_SF(0); }
                  break;
            }
         }
#undef ECM2_SF
      }
      else { ECM2_VERIFY(false, ERR_INTERNAL, "AFFINE qdata needs both integrators"); }
#undef ECM2_PF
#undef ECM2_PF_AF
      return;
   }
#define ECM2_PF_AF(V, AF)                                                                            \
   hipLaunchKernelGGL((k_apply_tpe_pf<D, Q, MASS, DIFF, SPLIT, V, AF>), grid, block, 0, s, a.ne,    \
                      a.blk_begin, a.blk_end, a.n_owned, a.gmap, a.qdd, a.qdm, a.x, a.xg, a.y, a.yg, b, rowtab, \
                      a.lane_flags, a.part, a.pslot)
#define ECM2_PF(V) ECM2_PF_AF(V, false)
   switch (var & 27)
   {
      case 0: ECM2_PF(0); break;
      case 1: ECM2_PF(1); break;
      case 2: ECM2_PF(2); break;
      case 3: ECM2_PF(3); break;
      case 8: ECM2_PF(8); break;
      case 9: ECM2_PF(9); break;
      case 16: ECM2_PF(16); break;
      case 17: ECM2_PF(17); break;
      default: ECM2_PF(0); break;
   }
#undef ECM2_PF
#undef ECM2_PF_AF
}

template <int D, int Q, bool MASS, bool DIFF>
void launch_tpe_mdq(const ApplyArgs &a, const Basis1D &b, const double *rowtab, hipStream_t s)
{
   const int nb = a.blk_end - a.blk_begin;
   if (nb <= 0) { return; }
   const int var = tpe_variant();
   ECM2_VERIFY(!a.part || a.lane_flags, ERR_INTERNAL, "partial-slot output needs the merge plan");
   ECM2_VERIFY(a.kind != QLAYOUT_AFFINE || a.lane_flags, ERR_INTERNAL, "AFFINE qdata needs the pipelined kernel");
   if (((var & 4) || a.part || a.kind == QLAYOUT_AFFINE) && a.lane_flags)
   {
      if (a.xg || a.yg) { launch_tpe_pf<D, Q, MASS, DIFF, true>(var, a, b, rowtab, s); }
      else { launch_tpe_pf<D, Q, MASS, DIFF, false>(var, a, b, rowtab, s); }
      return;
   }
   const dim3 grid((nb + 3) / 4), block(256);
   if (a.xg || a.yg)
   {
      hipLaunchKernelGGL((k_apply_tpe<D, Q, MASS, DIFF, true>), grid, block, 0, s, a.ne, a.blk_begin,
                         a.blk_end, a.n_owned, a.gmap, a.qdd, a.qdm, a.x, a.xg, a.y, a.yg, b, rowtab);
   }
   else
   {
      hipLaunchKernelGGL((k_apply_tpe<D, Q, MASS, DIFF, false>), grid, block, 0, s, a.ne, a.blk_begin,
                         a.blk_end, a.n_owned, a.gmap, a.qdd, a.qdm, a.x, a.xg, a.y, a.yg, b, rowtab);
   }
}

template <int D, int Q>
void launch_tpe_dq(bool mass, bool diff, const ApplyArgs &a, const Basis1D &b,
                   const double *rowtab, hipStream_t s)
{
   if (mass && diff) { launch_tpe_mdq<D, Q, true, true>(a, b, rowtab, s); }
   else if (mass) { launch_tpe_mdq<D, Q, true, false>(a, b, rowtab, s); }
   else if (diff) { launch_tpe_mdq<D, Q, false, true>(a, b, rowtab, s); }
}

int wpe_variant()
{
   static int v = [] {
      const char *e = std::getenv("ECM2_WPE_VARIANT");
      return e ? std::atoi(e) : 0;
   }();
   return v;
}

template <int D, int Q, bool MASS, bool DIFF>
void launch_wpe_mdq(const ApplyArgs &a, bool in_e, bool out_e, const Basis1D &b, hipStream_t s)
{
   constexpr int NQ = Q * Q * Q;
   const int nt = ((NQ + 63) / 64) * 64;
   const int e0 = a.blk_begin * 64, e1 = std::min(a.ne, a.blk_end * 64);
   if (e1 <= e0) { return; }
   const dim3 grid(e1 - e0), block(nt);
#define ECM2_WPE_LAUNCH(IE, OE)                                                                      \
   hipLaunchKernelGGL((k_apply_wpe<D, Q, MASS, DIFF, IE, OE>), grid, block, 0, s, a.pos, a.kind, a.ne, e0, \
                      a.n_owned, a.gmap, a.qdd, a.qdm, a.x, a.xg, a.y, a.yg, b, var)
   const int var = wpe_variant();
   if (in_e && out_e) { ECM2_WPE_LAUNCH(true, true); }
   else if (in_e) { ECM2_WPE_LAUNCH(true, false); }
   else if (out_e) { ECM2_WPE_LAUNCH(false, true); }
   else { ECM2_WPE_LAUNCH(false, false); }
#undef ECM2_WPE_LAUNCH
}

template <int D, int Q>
void launch_wpe_dq(bool mass, bool diff, const ApplyArgs &a, bool in_e, bool out_e,
                   const Basis1D &b, hipStream_t s)
{
   if (mass && diff) { launch_wpe_mdq<D, Q, true, true>(a, in_e, out_e, b, s); }
   else if (mass) { launch_wpe_mdq<D, Q, true, false>(a, in_e, out_e, b, s); }
   else if (diff) { launch_wpe_mdq<D, Q, false, true>(a, in_e, out_e, b, s); }
}

} // namespace

namespace kern
{

void coeff_gridfunc(int ne, int D, int Q, const int *gmap, const Basis1D &b, const CoeffDesc &c,
                    double *out, hipStream_t s)
{
   const long n = (long)ne * Q * Q * Q;
   if (n == 0) { return; }
   if (has_line(D, Q))
   {
      upload_basis(D, Q, b);
#define ECM2_COEFF_CASE(DD, QQ)                                                                      \
      if (D == DD && Q == QQ)                                                                        \
      {                                                                                              \
         hipLaunchKernelGGL((k_coeff_line<DD, QQ>), dim3(ne), dim3(64), 0, s, ne, gmap, c.lvec, c.scale, \
                            c.slope, c.t_ref, out);                                                  \
         ECM2_HIP(hipGetLastError());                                                                \
         return;                                                                                     \
      }
      ECM2_COEFF_CASE(2, 3) ECM2_COEFF_CASE(3, 4) ECM2_COEFF_CASE(4, 5) ECM2_COEFF_CASE(5, 6)
      ECM2_COEFF_CASE(6, 7) ECM2_COEFF_CASE(7, 8) ECM2_COEFF_CASE(2, 2) ECM2_COEFF_CASE(3, 3)
      ECM2_COEFF_CASE(4, 4) ECM2_COEFF_CASE(5, 5)
#undef ECM2_COEFF_CASE
   }
   hipLaunchKernelGGL(k_coeff_gridfunc, dim3(grid_for(n, 256)), dim3(256), 0, s, ne, D, Q, gmap,
                      b, c.lvec, c.scale, c.slope, c.t_ref, out);
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
                            enodes, W, b1, scm, scd, qd_diff, qd_mass);                                  \
      }                                                                                                  \
      else                                                                                               \
      {                                                                                                  \
         hipLaunchKernelGGL((k_setup_nodes_t<QQ, false>), dim3(grid_for(nb, 256)), dim3(256), 0, s, nullptr, L.ne, \
                            enodes, W, b1, scm, scd, qd_diff, qd_mass);                                  \
      }                                                                                                  \
      ECM2_HIP(hipGetLastError());                                                                       \
      return;                                                                                            \
   }
   ECM2_SETUP_CASE(2) ECM2_SETUP_CASE(3) ECM2_SETUP_CASE(4) ECM2_SETUP_CASE(5)
   ECM2_SETUP_CASE(6) ECM2_SETUP_CASE(7) ECM2_SETUP_CASE(8)
#undef ECM2_SETUP_CASE
   hipLaunchKernelGGL(k_setup_nodes, dim3(grid_for(n, 256)), dim3(256), 0, s, L.pos, L.kind, L.ne, Q,
                      enodes, W, b1, scm, scd, qd_diff, qd_mass);
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

void setup_affine(const QLayout &L, int Q, const double *enodes, const double *J, const double *W,
                  const CoeffDesc *cm, const CoeffDesc *cd, const double *cm_q, const double *cd_q,
                  double *qd_fac, double *qd_pair, hipStream_t s)
{
   if (L.ne == 0) { return; }
   ECM2_VERIFY(L.affine() && cm && cd, ERR_INTERNAL, "affine setup needs an AFFINE layout and both coefficients");
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
                            enodes, J, W, scm, scd, qd_fac, qd_pair);                                    \
      }                                                                                                  \
      else                                                                                               \
      {                                                                                                  \
         hipLaunchKernelGGL((k_setup_affine<QQ, false>), dim3(grid_for(n, 256)), dim3(256), 0, s, nullptr, L.ne, \
                            enodes, J, W, scm, scd, qd_fac, qd_pair);                                    \
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

void apply_tpe(int D, int Q, bool mass, bool diff, const ApplyArgs &a, const Basis1D &b,
               const double *rowtab, hipStream_t s)
{
   if (a.ne == 0) { return; }
   if (D == 2 && Q == 3) { launch_tpe_dq<2, 3>(mass, diff, a, b, rowtab, s); }
   else if (D == 3 && Q == 4) { launch_tpe_dq<3, 4>(mass, diff, a, b, rowtab, s); }
   else { ECM2_VERIFY(false, ERR_UNSUPPORTED, "no thread-per-element kernel for D1D=" << D << " Q1D=" << Q); }
   ECM2_HIP(hipGetLastError());
}

// experiment knob ECM2_LINE_VARIANT: bit 1 = load each element's qdata at the top of its
// iteration instead of prefetching it during the previous element; bit 8 = one element per
// wave (compile-time; needs ECM2_LINE_CHUNK=1); bit 32 = load qdata inside the z stage
constexpr int kDefaultLineVariant = 8;  // one element per wave, qdata prefetched at the top

int line_variant()
{
   static int v = [] {
      const char *e = std::getenv("ECM2_LINE_VARIANT");
      return e ? std::atoi(e) : kDefaultLineVariant;
   }();
   return v;
}

template <int D, int Q, bool MASS, bool DIFF>
void launch_line_mdq(const ApplyArgs &a, const Basis1D &b, hipStream_t s)
{
   ECM2_VERIFY(a.chunks && a.chunk_off, ERR_INTERNAL, "line kernel needs its chunk table");
   const int c0 = a.chunk_off[a.blk_begin], c1 = a.chunk_off[a.blk_end];
   if (c1 <= c0) { return; }
   const dim3 grid(c1 - c0), block(64);
#define ECM2_LINE(SP, V)                                                                                  \
   hipLaunchKernelGGL((k_apply_line<D, Q, MASS, DIFF, SP, V>), grid, block, 0, s, c0, c1, a.chunks, a.n_owned, \
                      a.gmap, a.qdd, a.qdm, a.x, a.xg, a.y, a.yg, b, a.part)
   const bool split = a.xg || a.yg;
   if (a.kind == QLAYOUT_AFFINE_E)  // bit 64: AFFINE_E qdata (default variant only)
   {
      if constexpr (MASS && DIFF)
      {
         if (line_variant() & 8) { if (split) { ECM2_LINE(true, 72); } else { ECM2_LINE(false, 72); } }
         else { if (split) { ECM2_LINE(true, 64); } else { ECM2_LINE(false, 64); } }
      }
      else { ECM2_VERIFY(false, ERR_INTERNAL, "AFFINE qdata needs both integrators"); }
      return;
   }
   switch (line_variant() & 46)
   {
      case 2: if (split) { ECM2_LINE(true, 2); } else { ECM2_LINE(false, 2); } break;
      case 8: if (split) { ECM2_LINE(true, 8); } else { ECM2_LINE(false, 8); } break;
      case 40: if (split) { ECM2_LINE(true, 40); } else { ECM2_LINE(false, 40); } break;
      case 32: if (split) { ECM2_LINE(true, 32); } else { ECM2_LINE(false, 32); } break;
      default: if (split) { ECM2_LINE(true, 0); } else { ECM2_LINE(false, 0); } break;
   }
#undef ECM2_LINE
}

template <int D, int Q>
void launch_line_dq(bool mass, bool diff, const ApplyArgs &a, const Basis1D &b, hipStream_t s)
{
   if (mass && diff) { launch_line_mdq<D, Q, true, true>(a, b, s); }
   else if (mass) { launch_line_mdq<D, Q, true, false>(a, b, s); }
   else if (diff) { launch_line_mdq<D, Q, false, true>(a, b, s); }
}

int line_chunk_limit() { return (line_variant() & 8) ? 1 : 8; }

bool has_line(int D, int Q)
{
   return (Q == D + 1 || Q == D) && D >= 2 && D <= 7 && Q <= 8;
}

void upload_basis(int D, int Q, const Basis1D &b)
{
   static std::mutex mu;
   static std::set<std::tuple<int, int, int>> done;  // (device, D, Q)
   int dev = 0;
   ECM2_HIP(hipGetDevice(&dev));
   std::lock_guard<std::mutex> lock(mu);
   if (!done.insert({dev, D, Q}).second) { return; }
   ECM2_VERIFY(D >= 1 && D <= MAX_D1D && Q >= 1 && Q <= MAX_Q1D, ERR_ARG, "basis size");
   ECM2_HIP(hipMemcpyToSymbol(HIP_SYMBOL(c_basis), &b, sizeof(Basis1D),
                              ((size_t)(D - 1) * MAX_Q1D + (Q - 1)) * sizeof(Basis1D), hipMemcpyHostToDevice));
}

// experiment knob ECM2_BRICK_VARIANT (bit 1: qdata loaded at the z stage; bit 2: 16-byte paired
// qdata loads, native layout; bit 4: one LDS buffer per element, AFFINE_E)
// default 8: XCD-contiguous brick order on AFFINE_E (C5: kernel 0.575 -> 0.566 ms, Mult
// 0.754 -> 0.739 ms, profiles/r1_ab_xcd_brick.txt); ECM2_BRICK_VARIANT=0: launch order
int brick_variant()
{
   static int v = [] {
      const char *e = std::getenv("ECM2_BRICK_VARIANT");
      return e ? std::atoi(e) : 8;
   }();
   return v;
}

template <int D, int Q, int BZ, bool MASS, bool DIFF>
void launch_brick_mdq(const ApplyArgs &a, hipStream_t s)
{
   const int k0 = a.brick_off[a.blk_begin], k1 = a.brick_off[a.blk_end];
   if (k1 <= k0) { return; }
   ECM2_VERIFY(a.part_brick, ERR_INTERNAL, "brick kernel needs its partial slots");
   const dim3 grid(k1 - k0), block(BrickShape<D, Q, BZ>::NT);
#define ECM2_BRICK(SP, V)                                                                               \
   hipLaunchKernelGGL((k_apply_brick<D, Q, BZ, MASS, DIFF, SP, V>), grid, block, 0, s, k0, k1, a.belem, \
                      a.bmap, a.n_owned, a.qdd, a.qdm, a.x, a.xg, a.y, a.yg, a.part_brick)
   const bool split = a.xg || a.yg;
   if (a.kind == QLAYOUT_AFFINE_E)  // bit 64: AFFINE_E qdata
   {
      if constexpr (MASS && DIFF)
      {
         switch (brick_variant() & 13)
         {
            case 8: if (split) { ECM2_BRICK(true, 320); } else { ECM2_BRICK(false, 320); } break;
            case 1: if (split) { ECM2_BRICK(true, 65); } else { ECM2_BRICK(false, 65); } break;
            case 4: if (split) { ECM2_BRICK(true, 192); } else { ECM2_BRICK(false, 192); } break;
            case 5: if (split) { ECM2_BRICK(true, 193); } else { ECM2_BRICK(false, 193); } break;
            default: if (split) { ECM2_BRICK(true, 64); } else { ECM2_BRICK(false, 64); } break;
         }
      }
      else { ECM2_VERIFY(false, ERR_INTERNAL, "AFFINE qdata needs both integrators"); }
      return;
   }
   switch (brick_variant() & 3)
   {
      case 1: if (split) { ECM2_BRICK(true, 1); } else { ECM2_BRICK(false, 1); } break;
      case 2: if (split) { ECM2_BRICK(true, 2); } else { ECM2_BRICK(false, 2); } break;
      default: if (split) { ECM2_BRICK(true, 0); } else { ECM2_BRICK(false, 0); } break;
   }
#undef ECM2_BRICK
}

template <int D, int Q, int BZ>
void launch_brick_dq(bool mass, bool diff, const ApplyArgs &a, hipStream_t s)
{
   if (mass && diff) { launch_brick_mdq<D, Q, BZ, true, true>(a, s); }
   else if (mass) { launch_brick_mdq<D, Q, BZ, true, false>(a, s); }
   else if (diff) { launch_brick_mdq<D, Q, BZ, false, true>(a, s); }
}

// bricks of 2 x 2 x bz elements for Q1D = D1D + 1 (the default rule), p = 3..6; a
// 2 x 2 x 2 brick's LDS (16 S doubles) exceeds 160 KiB at p = 6; column bricks (bz = 4, 8)
// march 2 x 2 layers and need one layer's LDS
bool has_brick(int D, int Q, int bz)
{
   if (Q != D + 1 || D < 4 || D > 7) { return false; }
   return bz == 1 || (bz == 2 && D <= 6) || bz == 4 || (bz == 8 && D == 5);
}

int brick_points(int D, int bz) { return (2 * D - 1) * (2 * D - 1) * (bz * (D - 1) + 1); }

static void apply_brick(int D, int Q, bool mass, bool diff, const ApplyArgs &a, hipStream_t s)
{
#define ECM2_BRICK_CASE(DD, BZ)                                         \
   if (D == DD && a.brick_bz == BZ)                                     \
   {                                                                    \
      launch_brick_dq<DD, DD + 1, BZ>(mass, diff, a, s);                \
      ECM2_HIP(hipGetLastError());                                      \
      return;                                                           \
   }
   ECM2_BRICK_CASE(4, 1)
   ECM2_BRICK_CASE(4, 2)
   ECM2_BRICK_CASE(5, 1)
   ECM2_BRICK_CASE(5, 2)
   ECM2_BRICK_CASE(6, 1)
   ECM2_BRICK_CASE(6, 2)
   ECM2_BRICK_CASE(7, 1)
   ECM2_BRICK_CASE(4, 4)  // column bricks: 2 x 2 x bz marched in z
   ECM2_BRICK_CASE(5, 4)
   ECM2_BRICK_CASE(5, 8)
   ECM2_BRICK_CASE(6, 4)
   ECM2_BRICK_CASE(7, 4)
#undef ECM2_BRICK_CASE
   ECM2_VERIFY(false, ERR_UNSUPPORTED, "no brick kernel for D1D=" << D << " Q1D=" << Q << " bz=" << a.brick_bz);
}

void apply_line(int D, int Q, bool mass, bool diff, const ApplyArgs &a, const Basis1D &b, hipStream_t s)
{
   if (a.ne == 0) { return; }
   if (a.brick_bz) { apply_brick(D, Q, mass, diff, a, s); }
#define ECM2_LINE_CASE(DD, QQ)                                        \
   if (D == DD && Q == QQ)                                            \
   {                                                                  \
      launch_line_dq<DD, QQ>(mass, diff, a, b, s);                    \
      ECM2_HIP(hipGetLastError());                                    \
      return;                                                         \
   }
   ECM2_LINE_CASE(2, 3)
   ECM2_LINE_CASE(3, 4)
   ECM2_LINE_CASE(4, 5)
   ECM2_LINE_CASE(5, 6)
   ECM2_LINE_CASE(6, 7)
   ECM2_LINE_CASE(7, 8)
   ECM2_LINE_CASE(2, 2)
   ECM2_LINE_CASE(3, 3)
   ECM2_LINE_CASE(4, 4)
   ECM2_LINE_CASE(5, 5)
#undef ECM2_LINE_CASE
   ECM2_VERIFY(false, ERR_UNSUPPORTED, "no line kernel for D1D=" << D << " Q1D=" << Q);
}

void apply_wpe(int D, int Q, bool mass, bool diff, const ApplyArgs &a, bool in_e, bool out_e,
               const Basis1D &b, hipStream_t s)
{
   if (a.ne == 0) { return; }
#define ECM2_WPE_CASE(DD, QQ)                                         \
   if (D == DD && Q == QQ)                                            \
   {                                                                  \
      launch_wpe_dq<DD, QQ>(mass, diff, a, in_e, out_e, b, s);        \
      ECM2_HIP(hipGetLastError());                                    \
      return;                                                         \
   }
   ECM2_WPE_CASE(2, 3)
   ECM2_WPE_CASE(3, 4)
   ECM2_WPE_CASE(4, 5)
   ECM2_WPE_CASE(5, 6)
   ECM2_WPE_CASE(2, 2)
   ECM2_WPE_CASE(3, 3)
   ECM2_WPE_CASE(4, 4)
   ECM2_WPE_CASE(5, 5)
   ECM2_WPE_CASE(6, 7)
#undef ECM2_WPE_CASE
   ECM2_VERIFY(false, ERR_UNSUPPORTED, "no PA kernel for D1D=" << D << " Q1D=" << Q);
}

void restriction_mult(long n, int nd, const int *gm, const double *x, double *xe, hipStream_t s)
{
   (void)nd;
   if (n == 0) { return; }
   hipLaunchKernelGGL(k_restriction_mult, dim3(grid_for(n, 256)), dim3(256), 0, s, n, gm, x, xe);
   ECM2_HIP(hipGetLastError());
}

void restriction_mult_transpose(int ndofs, int nd, const int *offsets, const int *indices,
                                const double *xe, double *y, hipStream_t s)
{
   (void)nd;
   if (ndofs == 0) { return; }
   hipLaunchKernelGGL(k_restriction_mult_transpose, dim3(grid_for(ndofs, 256)), dim3(256), 0, s,
                      ndofs, offsets, indices, xe, y);
   ECM2_HIP(hipGetLastError());
}

void diagonal(const int *pos, int D, int Q, int layout, int ne, const int *gm, const double *qdd,
              const double *qdm, double *diag, bool out_e, const Basis1D &b, hipStream_t s)
{
   const long n = (long)ne * D * D * D;
   if (n == 0) { return; }
   upload_basis(D, Q, b);
#define ECM2_DIAG_CASE(DD, QQ)                                                                             \
   if (D == DD && Q == QQ)                                                                                 \
   {                                                                                                       \
      hipLaunchKernelGGL((k_diag_sf<DD, QQ>), dim3(ne), dim3(64), 0, s, pos, layout, ne, gm, qdd, qdm, diag, \
                         out_e);                                                                           \
      ECM2_HIP(hipGetLastError());                                                                         \
      return;                                                                                              \
   }
   ECM2_DIAG_CASE(2, 3)
   ECM2_DIAG_CASE(3, 4)
   ECM2_DIAG_CASE(4, 5)
   ECM2_DIAG_CASE(5, 6)
   ECM2_DIAG_CASE(6, 7)
   ECM2_DIAG_CASE(7, 8)
   ECM2_DIAG_CASE(2, 2)
   ECM2_DIAG_CASE(3, 3)
   ECM2_DIAG_CASE(4, 4)
   ECM2_DIAG_CASE(5, 5)
#undef ECM2_DIAG_CASE
   hipLaunchKernelGGL(k_diagonal, dim3(grid_for(n, 128)), dim3(128), 0, s, pos, D, Q, layout, ne, gm,
                      qdd, qdm, diag, out_e, b);
   ECM2_HIP(hipGetLastError());
}

template <int D, int Q, bool MASS, bool DIFF>
static void launch_diag_tpe(const ApplyArgs &a, const Basis1D &b, const double *drow, hipStream_t s)
{
   const int nb = a.blk_end - a.blk_begin;
   if (nb <= 0) { return; }
   const dim3 grid((nb + 3) / 4), block(256);
#define ECM2_DIAG(SP, AF)                                                                               \
   if ((AF) && a.xwg == 8)                                                                              \
   {                                                                                                    \
      hipLaunchKernelGGL((k_diag_tpe<D, Q, MASS, DIFF, SP, AF, 8>), dim3((nb + 7) / 8), dim3(512), 0, s, a.ne, \
                         a.blk_begin, a.blk_end, a.n_owned, a.gmap, a.qdd, a.qdm, a.y, a.yg, b, drow,      \
                         a.lane_flags, a.part, a.pslot);                                                   \
   }                                                                                                    \
   else                                                                                                 \
   {                                                                                                    \
      hipLaunchKernelGGL((k_diag_tpe<D, Q, MASS, DIFF, SP, AF>), grid, block, 0, s, a.ne, a.blk_begin,    \
                         a.blk_end, a.n_owned, a.gmap, a.qdd, a.qdm, a.y, a.yg, b, drow, a.lane_flags,    \
                         a.part, a.pslot);                                                                 \
   }
   const bool aff = a.kind == QLAYOUT_AFFINE;
   ECM2_VERIFY(!aff || (MASS && DIFF), ERR_INTERNAL, "AFFINE qdata needs both integrators");
   if (a.yg) { if (aff) { ECM2_DIAG(true, true); } else { ECM2_DIAG(true, false); } }
   else { if (aff) { ECM2_DIAG(false, true); } else { ECM2_DIAG(false, false); } }
#undef ECM2_DIAG
}

template <int D, int Q>
static void launch_diag_tpe_dq(bool mass, bool diff, const ApplyArgs &a, const Basis1D &b, const double *drow,
                               hipStream_t s)
{
   if (mass && diff) { launch_diag_tpe<D, Q, true, true>(a, b, drow, s); }
   else if (mass) { launch_diag_tpe<D, Q, true, false>(a, b, drow, s); }
   else if (diff) { launch_diag_tpe<D, Q, false, true>(a, b, drow, s); }
}

void diagonal_tpe(int D, int Q, bool mass, bool diff, const ApplyArgs &a, const Basis1D &b, const double *drow,
                  hipStream_t s)
{
   if (a.ne == 0) { return; }
   if (D == 2 && Q == 3) { launch_diag_tpe_dq<2, 3>(mass, diff, a, b, drow, s); }
   else if (D == 3 && Q == 4) { launch_diag_tpe_dq<3, 4>(mass, diff, a, b, drow, s); }
   else { ECM2_VERIFY(false, ERR_UNSUPPORTED, "no thread-per-element diagonal for D1D=" << D << " Q1D=" << Q); }
   ECM2_HIP(hipGetLastError());
}

std::vector<double> make_diag_row_table(const DofToQuad &m)
{
   const int D = m.ndof, Q = m.nqpt, DD = D * D;
   std::vector<double> t((size_t)Q * Q * 6 * DD);
   for (int qz = 0; qz < Q; qz++)
      for (int qy = 0; qy < Q; qy++)
      {
         double *P = &t[(size_t)(qz * Q + qy) * 6 * DD];
         for (int dz = 0; dz < D; dz++)
            for (int dy = 0; dy < D; dy++)
            {
               const double By = m.B[qy + Q * dy], Gy = m.G[qy + Q * dy];
               const double Bz = m.B[qz + Q * dz], Gz = m.G[qz + Q * dz];
               const int o = dz * D + dy;
               P[0 * DD + o] = By * By * Bz * Bz;
               P[1 * DD + o] = Gy * Gy * Bz * Bz;
               P[2 * DD + o] = By * By * Gz * Gz;
               P[3 * DD + o] = Gy * By * Bz * Bz;
               P[4 * DD + o] = By * By * Gz * Bz;
               P[5 * DD + o] = Gy * By * Gz * Bz;
            }
      }
   return t;
}

void set_values(int n, const int *idx, double val, double *y, hipStream_t s)
{
   if (n == 0) { return; }
   hipLaunchKernelGGL(k_set_values, dim3(grid_for(n, 256)), dim3(256), 0, s, n, idx, val, y);
   ECM2_HIP(hipGetLastError());
}

void copy_values(int n, const int *idx, const double *x, double *y, hipStream_t s)
{
   if (n == 0) { return; }
   hipLaunchKernelGGL(k_copy_values, dim3(grid_for(n, 256)), dim3(256), 0, s, n, idx, x, y);
   ECM2_HIP(hipGetLastError());
}

void dot(int n, const double *a, const double *b, double *partials, double *out, hipStream_t s, double *hout)
{
   hipLaunchKernelGGL(k_dot_partial, dim3(kDotBlocks), dim3(256), 0, s, n, a, b, partials);
   hipLaunchKernelGGL(k_dot_final, dim3(1), dim3(256), 0, s, kDotBlocks, partials, out, hout);
   ECM2_HIP(hipGetLastError());
}

void pcg_update_xr(int n, const double *nom, const double *den, const double *d, const double *z,
                   double *x, double *r, hipStream_t s)
{
   hipLaunchKernelGGL(k_pcg_update_xr, dim3(grid_for(n, 256)), dim3(256), 0, s, n, nom, den, d, z, x, r);
   ECM2_HIP(hipGetLastError());
}

void pcg_step(int n, const double *nom, const double *den, const double *d, double *z, double *x, double *r,
              const double *dinv, double *partials, double *out, hipStream_t s, double *hout)
{
   hipLaunchKernelGGL(k_pcg_step, dim3(kDotBlocks), dim3(256), 0, s, n, nom, den, d, z, x, r, dinv, partials);
   hipLaunchKernelGGL(k_dot_final, dim3(1), dim3(256), 0, s, kDotBlocks, partials, out, hout);
   ECM2_HIP(hipGetLastError());
}

void ess_save_zero(int n, const int *idx, double *v, double *saved, hipStream_t s)
{
   if (n <= 0) { return; }
   hipLaunchKernelGGL(k_ess_save_zero, dim3(grid_for(n, 256)), dim3(256), 0, s, n, idx, v, saved);
   ECM2_HIP(hipGetLastError());
}

void ess_restore(int n, const int *idx, const double *saved, double *v, double *y, hipStream_t s)
{
   if (n <= 0) { return; }
   hipLaunchKernelGGL(k_ess_restore, dim3(grid_for(n, 256)), dim3(256), 0, s, n, idx, saved, v, y);
   ECM2_HIP(hipGetLastError());
}

void pcg_precond(int n, const double *dinv, const double *r, double *z, hipStream_t s)
{
   hipLaunchKernelGGL(k_pcg_precond, dim3(grid_for(n, 256)), dim3(256), 0, s, n, dinv, r, z);
   ECM2_HIP(hipGetLastError());
}

void pcg_update_d(int n, const double *betanom, const double *nom, const double *z, double *d,
                  hipStream_t s)
{
   hipLaunchKernelGGL(k_pcg_update_d, dim3(grid_for(n, 256)), dim3(256), 0, s, n, betanom, nom, z, d);
   ECM2_HIP(hipGetLastError());
}

void scale(int n, double a, double *y, hipStream_t s)
{
   if (n <= 0) { return; }
   hipLaunchKernelGGL(k_scale, dim3(grid_for(n, 256)), dim3(256), 0, s, n, a, y);
   ECM2_HIP(hipGetLastError());
}

void add_scaled(int n, const double *x, double c, const double *k, double *out, hipStream_t s)
{
   if (n <= 0) { return; }
   hipLaunchKernelGGL(k_add_scaled, dim3(grid_for(n, 256)), dim3(256), 0, s, n, x, c, k, out);
   ECM2_HIP(hipGetLastError());
}

void stream_copy(long n, const double *a, double *b, hipStream_t s)
{
   ECM2_VERIFY(n % 2 == 0 && ((uintptr_t)a % 16) == 0 && ((uintptr_t)b % 16) == 0, ERR_ARG,
               "stream_copy needs 16-byte aligned even-length arrays");
   hipLaunchKernelGGL(k_stream_copy, dim3(256 * 64), dim3(256), 0, s, n / 2, reinterpret_cast<const v2d *>(a),
                      reinterpret_cast<v2d *>(b));
   ECM2_HIP(hipGetLastError());
}

void reciprocal(int n, const double *a, double *out, hipStream_t s)
{
   if (n == 0) { return; }
   hipLaunchKernelGGL(k_reciprocal, dim3(grid_for(n, 256)), dim3(256), 0, s, n, a, out);
   ECM2_HIP(hipGetLastError());
}

void gather_idx(int n, const int *idx, const double *x, double *buf, hipStream_t s)
{
   if (n == 0) { return; }
   hipLaunchKernelGGL(k_gather_idx, dim3(grid_for(n, 256)), dim3(256), 0, s, n, idx, x, buf);
   ECM2_HIP(hipGetLastError());
}

void scatter_add_idx(int n, const int *idx, const double *buf, double *y, hipStream_t s)
{
   if (n == 0) { return; }
   hipLaunchKernelGGL(k_scatter_add_idx, dim3(grid_for(n, 256)), dim3(256), 0, s, n, idx, buf, y);
   ECM2_HIP(hipGetLastError());
}

void sum_partials(int i0, int i1, const int *dofs, const unsigned *meta, const int *slots, const double *part,
                  int n_owned, double *y, double *yg, hipStream_t s)
{
   if (i1 <= i0) { return; }
   // XCD-contiguous block order by default: +0.1-1.2% per Mult at C2 / C4 / C5, every pair of
   // profiles/r1_ab_sum_xcd.txt; ECM2_SUM_XCD=0 restores launch order
   static const bool xcd = [] {
      const char *e = std::getenv("ECM2_SUM_XCD");
      return !e || std::atoi(e) != 0;
   }();
   if (xcd)
   {
      hipLaunchKernelGGL(k_sum_partials<true>, dim3(grid_for(i1 - i0, 256)), dim3(256), 0, s, i0, i1, dofs, meta,
                         slots, part, n_owned, y, yg);
   }
   else
   {
      hipLaunchKernelGGL(k_sum_partials<false>, dim3(grid_for(i1 - i0, 256)), dim3(256), 0, s, i0, i1, dofs,
                         meta, slots, part, n_owned, y, yg);
   }
   ECM2_HIP(hipGetLastError());
}

void scatter_set_idx(int n, const int *idx, const double *buf, double *y, hipStream_t s)
{
   if (n == 0) { return; }
   hipLaunchKernelGGL(k_scatter_set_idx, dim3(grid_for(n, 256)), dim3(256), 0, s, n, idx, buf, y);
   ECM2_HIP(hipGetLastError());
}

std::vector<double> make_row_table(const DofToQuad &m)
{
   const int D = m.ndof, Q = m.nqpt, DD = D * D;
   std::vector<double> t((size_t)Q * Q * 3 * DD);
   for (int qz = 0; qz < Q; qz++)
      for (int qy = 0; qy < Q; qy++)
      {
         double *P = &t[(size_t)(qz * Q + qy) * 3 * DD];
         for (int dz = 0; dz < D; dz++)
            for (int dy = 0; dy < D; dy++)
            {
               const double By = m.B[qy + Q * dy], Gy = m.G[qy + Q * dy];
               const double Bz = m.B[qz + Q * dz], Gz = m.G[qz + Q * dz];
               P[0 * DD + dz * D + dy] = By * Bz;
               P[1 * DD + dz * D + dy] = Gy * Bz;
               P[2 * DD + dz * D + dy] = By * Gz;
            }
      }
   return t;
}

} // namespace kern
} // namespace ecm2
