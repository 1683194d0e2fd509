// k_line.hip -- fused apply for p >= 3 (line and brick kernels) and the sum-factorised
// diagonal (gfx950).
//
// Both apply kernels restate, per element, the reference's smem mass and diffusion kernels
// (bilininteg_mass_kernels.hpp:809-1033, bilininteg_diffusion_kernels.hpp:989-1214) as five
// 1D stages through LDS in which every active lane owns one 1D line of the current
// contraction direction in registers (a lane reads D or Q values from LDS once per Q or D
// multiply-adds; the reference reads two LDS operands per multiply-add), with the gather
// (ElementRestriction::Mult, restriction.cpp:109-129) and the scatter (MultTranspose,
// restriction.cpp:152-186) fused in.
#include "dev_common.hpp"

#include <algorithm>
#include <cstdlib>

namespace ecm2
{
namespace
{
using namespace dev;

// G: the qdata layout -- 0 the reference's native [e][6][NQ] / [e][NQ]; 1 AFFINE_E (per-element C
// and the point values (W beta, W alpha det J), or W beta alone without MASS); 2 TRILINEAR_E (the
// element's trilinear-map coefficients and the point values (W beta / det J, W alpha det J): D at
// the lane's points from J, as PADiffusionSetup3D, bilininteg_diffusion_kernels.cpp:349-362)
template <int D, int Q, bool MASS, bool DIFF, int G>
__device__ __forceinline__ void line_load_qdata(double (&qv)[7][Q], int e, int t,
                                                const double *__restrict__ qdd,
                                                const double *__restrict__ qdm, const QPts &qp)
{
   constexpr int NQ = Q * Q * Q, QQ = Q * Q;
   static_assert(G == 0 || DIFF, "compressed layouts carry the diffusion integrator");
   if (G != 0 && t < QQ)
   {
      double c[G == 1 ? 6 : 21];
#pragma unroll
      for (int k = 0; k < (G == 1 ? 6 : 21); k++) { c[k] = qdd[(size_t)e * (G == 1 ? 6 : 21) + k]; }
#pragma unroll
      for (int qz = 0; qz < Q; qz++)
      {
         const size_t eq = (size_t)e * NQ + qz * QQ + t;
         v2d p;
         if (MASS) { p = reinterpret_cast<const v2d *>(qdm)[eq]; }
         else { p = v2d{qdm[eq], 0.0}; }
         if (G == 1)
         {
#pragma unroll
            for (int k = 0; k < 6; k++) { qv[k][qz] = p.x * c[k]; }
         }
         else
         {
            double J[3][3], d[6];
            trilinear_jacobian(c, qp.x[t % Q], qp.x[t / Q], qp.x[qz], J);
            trilinear_dmat(J, p.x, d);
#pragma unroll
            for (int k = 0; k < 6; k++) { qv[k][qz] = d[k]; }
         }
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

// --------------------------------------------------------------------------
// Line kernel: one wave per element (the elements outside bricks), any (D, Q) with
// Q*Q <= 64 (p = 1..6), L-vectors in and out.  The z contraction, the quadrature-point
// weighting and the transposed z contraction are fused in registers on (qx, qy) lanes:
//   lanes (dy,dz): gather x-line, x-contract          -> s1 [2][dz][dy][qx]
//   lanes (qx,dz): y-contract                           -> s2 [3][dz][qy][qx]
//   lanes (qx,qy): z-contract, weight, z-transpose      -> s3 [3][dz][qy][qx]
//   lanes (qx,dz): y-transpose                          -> s4 [2][dz][dy][qx]
//   lanes (dy,dz): x-transpose, scatter
// The element's qdata is loaded at the top (in flight during the gather and the x / y
// stages).  gmap: [e][ND] encoded dof | shared << 30 | sign << 31; a shared dof goes to its
// partial slot part[e][a] (or, without partials, an atomic add); n_owned: dofs >= n_owned
// live in the ghost vectors xg / yg (distributed form; n_owned = ndofs otherwise).
// --------------------------------------------------------------------------
template <int D, int Q, bool MASS, bool DIFF, int G>
__global__ void __launch_bounds__(64)
k_apply_line(int c_begin, int c_end, const int *__restrict__ lelem, int n_owned, const int *__restrict__ gmap,
             const double *__restrict__ qdd, const double *__restrict__ qdm,
             const double *__restrict__ x, const double *__restrict__ xg,
             double *__restrict__ y, double *__restrict__ yg, const Basis1D *__restrict__ btab,
             double *__restrict__ part, const QPts qp)
{
   constexpr int ND = D * D * D, DD = D * D, QQ = Q * Q, DQ = D * Q;
   constexpr int SA = (2 * DD * Q > 3 * D * QQ) ? 2 * DD * Q : 3 * D * QQ;
   constexpr int SB = SA;
   static_assert(QQ <= 64, "line kernel needs Q1D <= 8");
   __shared__ double bufA[SA];  // s1, then s3
   __shared__ double bufB[SB];  // s2, then s4
   const int c = c_begin + (int)blockIdx.x;
   if (c >= c_end) { return; }  // whole wave
   const int t = threadIdx.x;
   const int e = lelem[c];

   double qv[7][Q];
   line_load_qdata<D, Q, MASS, DIFF, G>(qv, e, t, qdd, qdm, qp);
   // ---- lanes (dy, dz): gather the x-line, contract in x
   int gl[D];
   if (t < DD)
   {
      CBasis *bp = stage_basis(btab);
      const int *mp = gmap + (size_t)e * ND + t * D;
      double xl[D];
#pragma unroll
      for (int dx = 0; dx < D; dx++)
      {
         const int g = mp[dx];
         gl[dx] = g;
         const int d = bdof(g);
         const double v = d < n_owned ? x[d] : xg[d - n_owned];
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
      CBasis *bp = stage_basis(btab);
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
      CBasis *bp = stage_basis(btab);
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
   __syncthreads();
   // ---- lanes (qx, dz): transpose in y
   if (t < DQ)
   {
      CBasis *bp = stage_basis(btab);
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
            c2 += gy * l1[qy];   // -> B_x
            c2 += by * l2[qy];
         }
         bufB[(dz * D + dy) * Q + qx] = c1;
         bufB[DD * Q + (dz * D + dy) * Q + qx] = c2;
      }
   }
   __syncthreads();
   // ---- lanes (dy, dz): transpose in x, scatter
   if (t < DD)
   {
      CBasis *bp = stage_basis(btab);
      double l0[Q], l1[Q];
#pragma unroll
      for (int qx = 0; qx < Q; qx++)
      {
         l0[qx] = bufB[t * Q + qx];
         l1[qx] = bufB[DD * Q + t * Q + qx];
      }
#pragma unroll
      for (int dx = 0; dx < D; dx++)
      {
         double v = 0.0;
#pragma unroll
         for (int qx = 0; qx < Q; qx++) { v += bp->G[qx + MQ * dx] * l0[qx]; v += bp->B[qx + MQ * dx] * l1[qx]; }
         const int g = gl[dx];
         if (bneg(g)) { v = -v; }
         const int d = bdof(g);
         double *dst = d < n_owned ? y + d : yg + (d - n_owned);
         if (!bshared(g)) { *dst = v; }
         else if (part) { part[(size_t)e * ND + t * D + dx] = v; }
         else { unsafeAtomicAdd(dst, v); }
      }
   }
}

// --------------------------------------------------------------------------
// Brick kernel (p >= 3, both integrators): one workgroup per brick of 2 x 2 x BZ elements
// whose internal faces coincide (found by dof equality at setup, pa_form.cpp).  The five 1D
// stages of the line kernel run for all elements of the brick at once, lane = (element,
// line), so the 25 / 30 / 36-line stages of a p = 4 element fill 4-5 waves instead of
// leaving half of one wave idle.  The elements' outputs are then summed on the brick lattice
// ((2(D-1)+1)^2 (BZ(D-1)+1) points) in LDS in a fixed order, so the shared faces inside a
// brick never reach HBM: a lattice point held by this brick alone is plain-stored, one on
// the brick surface that other holders share goes to its partial slot
// part[brick][surface index] (face-grouped, brick_surface_index) for k_sum_partials
// (deterministic, no atomics).  Workgroups take bricks in XCD-contiguous order.
// G: 0 native qdata, 1 AFFINE_E (per-element C + one (W beta, W alpha det J) pair per point),
// 2 TRILINEAR_E (the element's trilinear-map coefficients + one (W beta / det J, W alpha det J)
// pair per point; the z stage evaluates J, adj(J) at its points).
// --------------------------------------------------------------------------
// Brick kernel layout and addressing (round 2; profiles/r2_ab_brick.txt: -8..-9% vs the
// round-1 form at C5):
//  * bank-conflict-free LDS images: every stage's lane -> element mapping starts each element
//    at a 32-lane boundary (x lines, y lines) or at a stride of S3 = QQ rounded up to 16 lanes
//    (z columns); the x-line image is [f][qx][dz][dy], the y/z image [g][dz][qy][qx] with a dz
//    stride DS = Q (mod 32) and an element stride SB = S3 (mod 32), so the lanes of a
//    ds_read_b64 group (32 lanes) / ds_write_b64 group (16 lanes) hit distinct banks in all
//    five stages (MI355X_MICROARCH.md §LDS);
//  * REG (lattice-numbered bricks, set up when every brick's map is d = base + X sx + Y sy +
//    Z sz and its shared points are exactly those on the brick faces other holders touch):
//    5 ints per brick (breg) replace the 405-entry lattice map, so the x gather is issued at
//    entry with no dependent map load, and the lattice stores compute their dofs;
//  * load order x gather -> qdata, branch-free: stage 1 waits for the gather only (vmcnt
//    counts in order), the qdata pairs stay in flight through the x and y stages.
// Measured and rejected: a persistent form prefetching the next brick's gather and qdata behind
// the z stage (155 VGPRs, 3 waves/SIMD: 0.83 vs 0.51 ms at C5).
// --------------------------------------------------------------------------
// One ds_read_b64 per value: the address goes through an opaque register copy, so the
// compiler cannot pair neighbouring reads into ds_read2_b64 (two accesses of 4 x 16 lanes on 32
// banks, 8 LDS cycles, against 2 x 2 for two ds_read_b64 on 64 banks; MI355X_MICROARCH.md §LDS).
typedef __attribute__((address_space(3))) const double lds_cdouble;
__device__ __forceinline__ double lds_read(const double *p)
{
   lds_cdouble *q = (lds_cdouble *)p;
   asm volatile("" : "+v"(q));
   return *q;
}

// ---- even/odd contractions (fe.hpp, BasisEO): a line x[D] is split into e[NE] (x_i + x_{D-1-i},
// then the middle value for odd D) and o[H] (x_i - x_{D-1-i}); a forward contraction computes
// the rows q < Q/2 and mirrors them; a transposed one accumulates into E[NE] / O[H] and merges.
typedef const __attribute__((address_space(4))) BasisEO CBasisEO;
__device__ __forceinline__ CBasisEO *stage_eo(const Basis1D *tab)
{
   CBasisEO *p = (CBasisEO *)&reinterpret_cast<const BasisDev *>(tab)->eo;
   asm volatile("" : "+s"(p));
   return p;
}
template <int D>
__device__ __forceinline__ void eo_split(const double (&x)[D], double (&e)[(D + 1) / 2], double (&o)[D / 2])
{
#pragma unroll
   for (int i = 0; i < D / 2; i++)
   {
      e[i] = x[i] + x[D - 1 - i];
      o[i] = x[i] - x[D - 1 - i];
   }
   if (D % 2) { e[D / 2] = x[D / 2]; }
}
// y = B x
template <int D, int Q>
__device__ __forceinline__ void eo_fwd_b(CBasisEO *t, const double (&e)[(D + 1) / 2], const double (&o)[D / 2],
                                         double (&y)[Q])
{
#pragma unroll
   for (int q = 0; q < (Q + 1) / 2; q++)
   {
      double s = 0.0, a = 0.0;
#pragma unroll
      for (int i = 0; i < (D + 1) / 2; i++) { s += t->BP[q + MQ * i] * e[i]; }
      if (2 * q + 1 == Q) { y[q] = s; }  // the middle row (odd Q): BM vanishes there
      else
      {
#pragma unroll
         for (int i = 0; i < D / 2; i++) { a += t->BM[q + MQ * i] * o[i]; }
         y[q] = s + a;
         y[Q - 1 - q] = s - a;
      }
   }
}
// y = G x
template <int D, int Q>
__device__ __forceinline__ void eo_fwd_g(CBasisEO *t, const double (&e)[(D + 1) / 2], const double (&o)[D / 2],
                                         double (&y)[Q])
{
#pragma unroll
   for (int q = 0; q < (Q + 1) / 2; q++)
   {
      double s = 0.0, a = 0.0;
#pragma unroll
      for (int i = 0; i < D / 2; i++) { s += t->GM[q + MQ * i] * o[i]; }
      if (2 * q + 1 == Q) { y[q] = s; }  // GP vanishes on the middle row
      else
      {
#pragma unroll
         for (int i = 0; i < (D + 1) / 2; i++) { a += t->GP[q + MQ * i] * e[i]; }
         y[q] = s + a;
         y[Q - 1 - q] = s - a;
      }
   }
}
// E, O += split of B^T y
template <int D, int Q>
__device__ __forceinline__ void eo_acc_bt(CBasisEO *t, const double (&y)[Q], double (&E)[(D + 1) / 2],
                                          double (&O)[D / 2])
{
#pragma unroll
   for (int q = 0; q < (Q + 1) / 2; q++)
   {
      if (2 * q + 1 == Q)
      {
#pragma unroll
         for (int i = 0; i < (D + 1) / 2; i++) { E[i] += t->BP[q + MQ * i] * y[q]; }
      }
      else
      {
         const double ye = y[q] + y[Q - 1 - q], yo = y[q] - y[Q - 1 - q];
#pragma unroll
         for (int i = 0; i < (D + 1) / 2; i++) { E[i] += t->BP[q + MQ * i] * ye; }
#pragma unroll
         for (int i = 0; i < D / 2; i++) { O[i] += t->BM[q + MQ * i] * yo; }
      }
   }
}
// E, O += split of G^T y
template <int D, int Q>
__device__ __forceinline__ void eo_acc_gt(CBasisEO *t, const double (&y)[Q], double (&E)[(D + 1) / 2],
                                          double (&O)[D / 2])
{
#pragma unroll
   for (int q = 0; q < (Q + 1) / 2; q++)
   {
      if (2 * q + 1 == Q)
      {
#pragma unroll
         for (int i = 0; i < D / 2; i++) { O[i] += t->GM[q + MQ * i] * y[q]; }
      }
      else
      {
         const double ye = y[q] + y[Q - 1 - q], yo = y[q] - y[Q - 1 - q];
#pragma unroll
         for (int i = 0; i < (D + 1) / 2; i++) { E[i] += t->GP[q + MQ * i] * yo; }
#pragma unroll
         for (int i = 0; i < D / 2; i++) { O[i] += t->GM[q + MQ * i] * ye; }
      }
   }
}
template <int D>
__device__ __forceinline__ void eo_zero(double (&E)[(D + 1) / 2], double (&O)[D / 2])
{
#pragma unroll
   for (int i = 0; i < (D + 1) / 2; i++) { E[i] = 0.0; }
#pragma unroll
   for (int i = 0; i < D / 2; i++) { O[i] = 0.0; }
}
template <int D>
__device__ __forceinline__ double eo_at(const double (&E)[(D + 1) / 2], const double (&O)[D / 2], int d)
{
   // d is a compile-time index after unrolling
   if (d < D / 2) { return E[d] + O[d]; }
   if (2 * d + 1 == D) { return E[(D - 1) / 2]; }  // odd D: the middle
   return E[D - 1 - d] - O[D - 1 - d];
}

template <int D, int Q, int BZ>
struct BrickShapeC
{
   static constexpr int NE = 4 * BZ, DD = D * D, QQ = Q * Q, DQ = D * Q, ND = D * D * D;
   static constexpr int LX = 2 * (D - 1) + 1, LY = LX, LZ = BZ * (D - 1) + 1, NB = LX * LY * LZ;
   static constexpr int SURF = brick_surface_points(D, BZ);
   static constexpr int L2S = (DQ > DD ? DQ : DD) <= 32 ? 32 : 64;  // lanes per element, line stages
   static constexpr int S3 = ((QQ + 15) / 16) * 16;                 // lanes per element, z stage
   static constexpr int DS = (QQ <= Q + 32 * ((QQ - Q + 31) / 32)) ? Q + 32 * ((QQ - Q + 31) / 32) : QQ;
   static constexpr int SA = 2 * DD * Q;                            // x-line image per element
   static constexpr int SB0 = 3 * D * DS > ND ? 3 * D * DS : ND;
   static constexpr int SB = SB0 + ((S3 % 32) - (SB0 % 32) + 32) % 32;  // SB = S3 (mod 32)
   static constexpr int NTL = NE * L2S, NT3 = NE * S3;
   static constexpr int NT = (((NTL > NT3 ? NTL : NT3) + 63) / 64) * 64;
   static constexpr int WPE = (D <= 5 && BZ == 1) ? 4 : 1;
};

// faces of the brick lattice containing point (X, Y, Z): bits X = 0, X = LX-1, Y = 0, ...
template <int LX, int LY, int LZ>
__host__ __device__ constexpr int brick_faces(int X, int Y, int Z)
{
   return (X == 0) | (X == LX - 1) << 1 | (Y == 0) << 2 | (Y == LY - 1) << 3 | (Z == 0) << 4 | (Z == LZ - 1) << 5;
}

// Lattice-point table of the brick kernel's final stage (round 3), the same for every brick of
// a (D, BZ): per lattice point p (X fastest) the LDS offsets of its holders' outputs in the
// element-output image [e][dx][dz][dy], in ascending element order and padded with the image's
// zero slot (NE SB), two 16-bit offsets per int; then X | Y << 8 | Z << 16 | faces << 24; then
// the point's surface index (brick_surface_index, -1 inside).  A thread reads its points' rows
// once and sums 4 (8) LDS values per point with no per-point index arithmetic: the loop it
// replaces derived the holder set per point (variable-trip loops over the candidate elements)
// and was ~22% of the kernel's VALU instructions at p = 4.
template <int D, int Q, int BZ>
struct BrickPtTable
{
   using S = BrickShapeC<D, Q, BZ>;
   static constexpr int NH = 4 * BZ, NW = NH / 2 + 2;
   int w[S::NB][NW];
   constexpr BrickPtTable() : w()
   {
      for (int p = 0; p < S::NB; p++)
      {
         const int X = p % S::LX, Y = (p / S::LX) % S::LY, Z = p / (S::LX * S::LY);
         int off[NH] = {};
         int n = 0;
         // holders along one direction: P < D-1 -> element 0 at P; P == D-1 -> elements 0 (D-1)
         // and 1 (0); P > D-1 -> element 1 at P - (D-1)
         const int nz = BZ == 2 && Z == D - 1 ? 2 : 1, ny = Y == D - 1 ? 2 : 1, nx = X == D - 1 ? 2 : 1;
         for (int iz = 0; iz < nz; iz++)
            for (int iy = 0; iy < ny; iy++)
               for (int ix = 0; ix < nx; ix++)
               {
                  const int cx = X < D - 1 ? 0 : (X == D - 1 ? ix : 1), lx = cx == 0 ? X : X - (D - 1);
                  const int cy = Y < D - 1 ? 0 : (Y == D - 1 ? iy : 1), ly = cy == 0 ? Y : Y - (D - 1);
                  const int cz = BZ == 1 ? 0 : (Z < D - 1 ? 0 : (Z == D - 1 ? iz : 1)), lz = cz == 0 ? Z : Z - (D - 1);
                  const int elt = cx + 2 * (cy + 2 * cz);
                  off[n++] = elt * S::SB + lx * S::DD + lz * D + ly;
               }
         for (; n < NH; n++) { off[n] = S::NE * S::SB; }
         for (int h = 0; h < NH / 2; h++) { w[p][h] = off[2 * h] | off[2 * h + 1] << 16; }
         w[p][NH / 2] = X | Y << 8 | Z << 16 | brick_faces<S::LX, S::LY, S::LZ>(X, Y, Z) << 24;
         w[p][NH / 2 + 1] = brick_surface_index(D, BZ, X, Y, Z);
      }
   }
};
template <int D, int Q, int BZ>
__device__ const BrickPtTable<D, Q, BZ> kBrickPts = BrickPtTable<D, Q, BZ>();

// Waves per SIMD a brick kernel is built for: the TRILINEAR_E z stage's column geometry takes it
// past 128 VGPRs (8 values spilled at 4 waves); at 3 waves it holds 140 without spills
// (profiles/r4/ab_bw3.txt: kernel -1%).
template <int D, int Q, int BZ, int G>
constexpr int brick_wpe()
{
   constexpr int W = BrickShapeC<D, Q, BZ>::WPE;
   return (G == 2 && W > 3) ? 3 : W;
}
template <int D, int Q, int BZ, bool SPLIT, int G, bool REG>
__global__ void __launch_bounds__((BrickShapeC<D, Q, BZ>::NT), (brick_wpe<D, Q, BZ, G>()))
k_apply_brick_c(int k_begin, int k_end, const int *__restrict__ belem, const int *__restrict__ bmap,
                const int *__restrict__ breg, int n_owned, const double *__restrict__ qdd,
                const double *__restrict__ qdm, const double *__restrict__ x, const double *__restrict__ xg,
                double *__restrict__ y, double *__restrict__ yg, const Basis1D *__restrict__ btab,
                double *__restrict__ part, const QPts qp)
{
   // G: 0 per-point qdata, 1 AFFINE_E, 2 TRILINEAR_E, 3 AFFINE_E with every C diagonal (axis-aligned elements:
   // the general product's values, whose off-diagonal terms would add exact zeros)
   constexpr bool AFF = G != 0;  // a compressed layout: point pairs + per-element data
   using S = BrickShapeC<D, Q, BZ>;
   constexpr int NE = S::NE, DD = S::DD, QQ = S::QQ, DQ = S::DQ, SA = S::SA, SB = S::SB, DS = S::DS;
   constexpr int LX = S::LX, LY = S::LY, NB = S::NB, L2S = S::L2S, S3 = S::S3, NQ = Q * Q * Q;
   constexpr int NEO = (D + 1) / 2, NOO = D / 2;  // even / odd parts of a split line
   static_assert(QQ <= 64, "brick kernel needs Q1D <= 8");
   static_assert(DQ <= L2S && DD <= L2S, "line stages: one lane per line");
   static_assert(!(REG && SPLIT), "regular bricks address one L-vector");
   __shared__ double sXL[NE * SA];      // x lines: [e][f][qx][dz][dy]
   __shared__ double sYQ[NE * SB + 1];  // y / z planes: [e][g][dz (stride DS)][qy][qx]; then outputs [e][dx][dz][dy]; zero slot
   const int k = k_begin + xcd_contiguous(blockIdx.x, gridDim.x);
   if (k >= k_end) { return; }  // whole workgroup
   const int t = threadIdx.x;
   if (t == 0) { sYQ[NE * SB] = 0.0; }  // the point table's padding slot (published by the first barrier)
   const int eL = t / L2S, lL = t % L2S;                 // line stages
   const bool actL = eL < NE && lL < DD;                 // stages 1, 5: lL = dy + D dz
   const bool act2 = eL < NE && lL < DQ;                 // stages 2, 4
   const int e3 = t / S3, l3 = t % S3;                   // z stage: l3 = qx + Q qy
   const bool act3 = e3 < NE && l3 < QQ;
   int base = 0, sx = 0, sy = 0, sz = 0, mask = 0;
   if (REG)
   {
      const int *r = breg + (size_t)k * 8;  // workgroup-uniform: scalar loads
      base = r[0]; sx = r[1]; sy = r[2]; sz = r[3]; mask = r[4];
   }
   const int *bm = bmap + (size_t)k * NB;
   auto lattice = [&](int elt, int dx, int dy, int dz) {
      const int ex = elt & 1, ey = (elt >> 1) & 1, ez = elt >> 2;
      return ((ez * (D - 1) + dz) * LY + ey * (D - 1) + dy) * LX + ex * (D - 1) + dx;
   };

   // ---- loads, branch-free: element ids, the x-line gather, then this lane's z-stage qdata (in
   // flight through stages 1-2).  Loads under a branch leave the compiler's wait counts unknown
   // at the join, and it then waits for all of them (the x stage would wait for the qdata);
   // idle lanes load a neighbour's (clamped) addresses instead and ignore the values.
   const int eLc = eL < NE ? eL : NE - 1, lLc = lL < DD ? lL : DD - 1;
   const int e = belem[(size_t)k * NE + (e3 < NE ? e3 : NE - 1)];
   const int l3c = l3 < QQ ? l3 : QQ - 1;
   double xl[D];
   {
      const int dy = lLc % D, dz = lLc / D, ex = eLc & 1, ey = (eLc >> 1) & 1, ez = eLc >> 2;
      if (REG)
      {
         const int d0 = base + (ex * (D - 1)) * sx + (ey * (D - 1) + dy) * sy + (ez * (D - 1) + dz) * sz;
#pragma unroll
         for (int dx = 0; dx < D; dx++) { xl[dx] = x[d0 + dx * sx]; }
      }
      else
      {
         const int *mp = bm + lattice(eLc, 0, dy, dz);
#pragma unroll
         for (int dx = 0; dx < D; dx++)
         {
            const int d = bdof(mp[dx]);
            xl[dx] = (!SPLIT || d < n_owned) ? x[d] : xg[d - n_owned];
         }
      }
   }
   __builtin_amdgcn_sched_barrier(0);  // keep the gather ahead of the qdata loads
   double qv[7][Q];
   v2d pa[Q];
   double cc[6];
   if (AFF)
   {
      // the point pairs are streamed once per Mult: nontemporal, so they do not evict the x lines
      // neighbouring bricks gather again (profiles/r3_ab_bnt.txt: kernel -1%, Mult -2%)
#pragma unroll
      for (int qz = 0; qz < Q; qz++)
      {
         pa[qz] = __builtin_nontemporal_load(reinterpret_cast<const v2d *>(qdm) + (size_t)e * NQ + qz * QQ + l3c);
      }
#pragma unroll
      for (int c = 0; c < (G == 1 ? 6 : 0); c++) { cc[c] = qdd[(size_t)e * 6 + c]; }
      if (G == 3)
      {
         cc[0] = qdd[(size_t)e * 6];
         cc[3] = qdd[(size_t)e * 6 + 3];
         cc[5] = qdd[(size_t)e * 6 + 5];
      }
   }
   else { line_load_qdata<D, Q, true, true, 0>(qv, e, l3c, qdd, qdm, qp); }

   // ---- lanes (element, dy, dz): contract in x -> sXL [f][qx][l]
   if (actL)
   {
      double *o = sXL + eL * SA + lL;
      CBasisEO *te = stage_eo(btab);
      double xe[NEO], xo[NOO], u[Q], v[Q];
      eo_split<D>(xl, xe, xo);
      eo_fwd_b<D, Q>(te, xe, xo, u);
      eo_fwd_g<D, Q>(te, xe, xo, v);
#pragma unroll
      for (int qx = 0; qx < Q; qx++)
      {
         o[qx * DD] = u[qx];
         o[Q * DD + qx * DD] = v[qx];
      }
   }
   if (k_begin < 0)  // never: a use outside the x stage stops the gather sinking behind the qdata
   {
      double u = 0.0;
#pragma unroll
      for (int dx = 0; dx < D; dx++) { u += xl[dx]; }
      part[t] = u;
   }
   __syncthreads();
   // ---- lanes (element, qx, dz), l2 = qx + Q dz: contract in y -> sYQ [g][dz][qy][qx]
   if (act2)
   {
      const int qx = lL % Q, dz = lL / Q;
      const double *in = sXL + eL * SA + qx * DD + dz * D;
      double la[D], lb[D];
#pragma unroll
      for (int dy = 0; dy < D; dy++)
      {
         la[dy] = lds_read(in + dy);
         lb[dy] = lds_read(in + Q * DD + dy);
      }
      double *o = sYQ + eL * SB + dz * DS + qx;
      CBasisEO *te = stage_eo(btab);
      double ae[NEO], ao[NOO], be[NEO], bo[NOO], gb[Q], bg[Q], bb[Q];
      eo_split<D>(la, ae, ao);
      eo_split<D>(lb, be, bo);
      eo_fwd_b<D, Q>(te, be, bo, gb);  // G_x B_y
      eo_fwd_g<D, Q>(te, ae, ao, bg);  // B_x G_y
      eo_fwd_b<D, Q>(te, ae, ao, bb);  // B_x B_y
#pragma unroll
      for (int qy = 0; qy < Q; qy++)
      {
         o[qy * Q] = gb[qy];
         o[D * DS + qy * Q] = bg[qy];
         o[2 * D * DS + qy * Q] = bb[qy];
      }
   }
   __syncthreads();
   // ---- lanes (element, qx, qy): contract in z, weight, transpose in z (in place)
   if (act3)
   {
      double *io = sYQ + e3 * SB + l3;
      double l0[D], l1[D], l2[D];
#pragma unroll
      for (int dz = 0; dz < D; dz++)
      {
         l0[dz] = lds_read(io + dz * DS);
         l1[dz] = lds_read(io + D * DS + dz * DS);
         l2[dz] = lds_read(io + 2 * D * DS + dz * DS);
      }
      // TRILINEAR_E: the column's Jacobian pieces, J[i][0] = a0 + b0 zeta, J[i][1] = a1 + b1 zeta,
      // J[i][2] = j2 (dev_common.hpp trilinear_jacobian at xi = x_qx, eta = x_qy)
      double a0[3], b0[3], a1[3], b1[3], j2[3];
      if (G == 2)
      {
         // the coefficients are read here (L2: the brick's four elements share 672 B), not with the
         // point pairs at entry, where 42 more live registers through stages 1-2 spill
         const double xi = qp.x[l3 % Q], et = qp.x[l3 / Q];
         const double *c = qdd + (size_t)e * 21;
#pragma unroll
         for (int i = 0; i < 3; i++)
         {
            a0[i] = c[i] + c[9 + i] * et;
            b0[i] = c[12 + i] + c[18 + i] * et;
            a1[i] = c[3 + i] + c[9 + i] * xi;
            b1[i] = c[15 + i] + c[18 + i] * xi;
            j2[i] = (c[6 + i] + c[12 + i] * xi) + b1[i] * et;
         }
      }
      // the quadrature-point operator: (f, m) = (W beta C grad u, W alpha det J u) at qz
      auto qpoint = [&](int qz, double gx, double gy, double gz, double u, double &fx, double &fy, double &fz,
                        double &m) {
         if (G == 2)
         {
            // f = (W beta / det J) adj(J) (adj(J)^T g), adj(J) from J at (x_qx, x_qy, x_qz)
            const double zt = qp.x[qz];
            double J[3][3], A[3][3];
#pragma unroll
            for (int i = 0; i < 3; i++)
            {
               J[i][0] = a0[i] + b0[i] * zt;
               J[i][1] = a1[i] + b1[i] * zt;
               J[i][2] = j2[i];
            }
            adj3(J, A);
            const double sc = pa[qz].x;
            double t0 = A[0][0] * gx, t1 = A[0][1] * gx, t2 = A[0][2] * gx;
            t0 += A[1][0] * gy; t1 += A[1][1] * gy; t2 += A[1][2] * gy;
            t0 += A[2][0] * gz; t1 += A[2][1] * gz; t2 += A[2][2] * gz;
            t0 *= sc; t1 *= sc; t2 *= sc;
            fx = A[0][0] * t0; fx += A[0][1] * t1; fx += A[0][2] * t2;
            fy = A[1][0] * t0; fy += A[1][1] * t1; fy += A[1][2] * t2;
            fz = A[2][0] * t0; fz += A[2][1] * t1; fz += A[2][2] * t2;
            m = pa[qz].y * u;
         }
         else if (G == 3)
         {
            const double wb = pa[qz].x;
            fx = wb * (cc[0] * gx);
            fy = wb * (cc[3] * gy);
            fz = wb * (cc[5] * gz);
            m = pa[qz].y * u;
         }
         else if (AFF)
         {
            const double wb = pa[qz].x;
            fx = wb * (cc[0] * gx + cc[1] * gy + cc[2] * gz);
            fy = wb * (cc[1] * gx + cc[3] * gy + cc[4] * gz);
            fz = wb * (cc[2] * gx + cc[4] * gy + cc[5] * gz);
            m = pa[qz].y * u;
         }
         else
         {
            fx = qv[0][qz] * gx + qv[1][qz] * gy + qv[2][qz] * gz;
            fy = qv[1][qz] * gx + qv[3][qz] * gy + qv[4][qz] * gz;
            fz = qv[2][qz] * gx + qv[4][qz] * gy + qv[5][qz] * gz;
            m = qv[6][qz] * u;
         }
      };
      // rows qz and Q-1-qz together: forward split contractions, the operator at both points, the
      // transposed contractions accumulated into split sums
      CBasisEO *te = stage_eo(btab);
      double e0[NEO], o0[NOO], e1[NEO], o1[NOO], e2[NEO], o2[NOO];
      eo_split<D>(l0, e0, o0);
      eo_split<D>(l1, e1, o1);
      eo_split<D>(l2, e2, o2);
      double A1E[NEO], A1O[NOO], A2E[NEO], A2O[NOO], A3E[NEO], A3O[NOO];
      eo_zero<D>(A1E, A1O);
      eo_zero<D>(A2E, A2O);
      eo_zero<D>(A3E, A3O);
#pragma unroll
      for (int qp = 0; qp < (Q + 1) / 2; qp++)
      {
         const int qr = Q - 1 - qp;
         const bool mid = qr == qp;
         double sx_ = 0.0, sy_ = 0.0, su = 0.0, sg = 0.0, ax = 0.0, ay = 0.0, au = 0.0, ag = 0.0;
#pragma unroll
         for (int i = 0; i < NEO; i++)
         {
            const double b = te->BP[qp + MQ * i];
            sx_ += b * e0[i];
            sy_ += b * e1[i];
            su += b * e2[i];
            if (!mid) { ag += te->GP[qp + MQ * i] * e2[i]; }
         }
#pragma unroll
         for (int i = 0; i < NOO; i++)
         {
            sg += te->GM[qp + MQ * i] * o2[i];
            if (!mid)
            {
               const double b = te->BM[qp + MQ * i];
               ax += b * o0[i];
               ay += b * o1[i];
               au += b * o2[i];
            }
         }
         double fxp, fyp, fzp, mp;
         qpoint(qp, sx_ + ax, sy_ + ay, sg + ag, su + au, fxp, fyp, fzp, mp);
         if (mid)
         {
#pragma unroll
            for (int i = 0; i < NEO; i++)
            {
               const double b = te->BP[qp + MQ * i];
               A1E[i] += b * fxp;
               A2E[i] += b * fyp;
               A3E[i] += b * mp;
            }
#pragma unroll
            for (int i = 0; i < NOO; i++) { A3O[i] += te->GM[qp + MQ * i] * fzp; }
         }
         else
         {
            double fxr, fyr, fzr, mr;
            qpoint(qr, sx_ - ax, sy_ - ay, sg - ag, su - au, fxr, fyr, fzr, mr);
            const double fxe = fxp + fxr, fxo = fxp - fxr, fye = fyp + fyr, fyo = fyp - fyr;
            const double fze = fzp + fzr, fzo = fzp - fzr, me = mp + mr, mo = mp - mr;
#pragma unroll
            for (int i = 0; i < NEO; i++)
            {
               const double b = te->BP[qp + MQ * i];
               A1E[i] += b * fxe;
               A2E[i] += b * fye;
               A3E[i] += b * me;
               A3E[i] += te->GP[qp + MQ * i] * fzo;
            }
#pragma unroll
            for (int i = 0; i < NOO; i++)
            {
               const double b = te->BM[qp + MQ * i];
               A1O[i] += b * fxo;
               A2O[i] += b * fyo;
               A3O[i] += b * mo;
               A3O[i] += te->GM[qp + MQ * i] * fze;
            }
         }
      }
#pragma unroll
      for (int dz = 0; dz < D; dz++)
      {
         io[dz * DS] = eo_at<D>(A1E, A1O, dz);
         io[D * DS + dz * DS] = eo_at<D>(A2E, A2O, dz);
         io[2 * D * DS + dz * DS] = eo_at<D>(A3E, A3O, dz);
      }
   }
   __syncthreads();
   // ---- lanes (element, dz, qx), l4 = dz + D qx: transpose in y -> sXL [f][qx][dz][dy]
   if (act2)
   {
      const int dz = lL % D, qx = lL / D;
      const double *in = sYQ + eL * SB + dz * DS + qx;
      double t0[Q], t1[Q], t2[Q];
#pragma unroll
      for (int qy = 0; qy < Q; qy++)
      {
         t0[qy] = lds_read(in + qy * Q);
         t1[qy] = lds_read(in + D * DS + qy * Q);
         t2[qy] = lds_read(in + 2 * D * DS + qy * Q);
      }
      double *o = sXL + eL * SA + qx * DD + dz * D;
      CBasisEO *te = stage_eo(btab);
      double C1E[NEO], C1O[NOO], C2E[NEO], C2O[NOO];
      eo_zero<D>(C1E, C1O);
      eo_zero<D>(C2E, C2O);
      eo_acc_bt<D, Q>(te, t0, C1E, C1O);
      eo_acc_gt<D, Q>(te, t1, C2E, C2O);
      eo_acc_bt<D, Q>(te, t2, C2E, C2O);
#pragma unroll
      for (int dy = 0; dy < D; dy++)
      {
         o[dy] = eo_at<D>(C1E, C1O, dy);
         o[Q * DD + dy] = eo_at<D>(C2E, C2O, dy);
      }
   }
   __syncthreads();
   // this thread's lattice points of the final stage: table rows (and map entries) issued here,
   // so their latency overlaps the x transpose
   using PT = BrickPtTable<D, Q, BZ>;
   constexpr int NIT = (NB + S::NT - 1) / S::NT, NW = PT::NW;
   int pw[NIT][NW], pg[NIT];
#pragma unroll
   for (int i = 0; i < NIT; i++)
   {
      const int p = t + i * S::NT < NB ? t + i * S::NT : NB - 1;
      const int *row = kBrickPts<D, Q, BZ>.w[p];
#pragma unroll
      for (int j = 0; j < NW; j++) { pw[i][j] = row[j]; }
      pg[i] = REG ? 0 : bm[p];
   }
   // ---- lanes (element, dy, dz): transpose in x -> element outputs [e][dx][dz][dy] in sYQ
   if (actL)
   {
      const double *in = sXL + eL * SA + lL;
      double l0[Q], l1[Q];
#pragma unroll
      for (int qx = 0; qx < Q; qx++)
      {
         l0[qx] = lds_read(in + qx * DD);
         l1[qx] = lds_read(in + Q * DD + qx * DD);
      }
      CBasisEO *te = stage_eo(btab);
      double VE[NEO], VO[NOO];
      eo_zero<D>(VE, VO);
      eo_acc_gt<D, Q>(te, l0, VE, VO);
      eo_acc_bt<D, Q>(te, l1, VE, VO);
#pragma unroll
      for (int dx = 0; dx < D; dx++) { sYQ[eL * SB + dx * DD + lL] = eo_at<D>(VE, VO, dx); }
   }
   __syncthreads();
   // ---- lattice points: sum the holders in ascending element order (the (z, y, x) order of
   // the point table), store or publish
#pragma unroll
   for (int i = 0; i < NIT; i++)
   {
      if (NB % S::NT != 0 && i == NIT - 1 && t + i * S::NT >= NB) { break; }
      double v = sYQ[pw[i][0] & 0xffff];
      v += sYQ[pw[i][0] >> 16];
#pragma unroll
      for (int h = 1; h < NW - 2; h++)
      {
         v += sYQ[pw[i][h] & 0xffff];
         v += sYQ[pw[i][h] >> 16];
      }
      const int c = pw[i][NW - 2];
      int d;
      bool shared;
      if (REG)
      {
         d = base + (c & 255) * sx + ((c >> 8) & 255) * sy + ((c >> 16) & 255) * sz;
         shared = ((c >> 24) & mask) != 0;
      }
      else
      {
         d = bdof(pg[i]);
         shared = bshared(pg[i]);
      }
      if (!shared) { *((!SPLIT || d < n_owned) ? y + d : yg + (d - n_owned)) = v; }
      else { part[(size_t)k * S::SURF + pw[i][NW - 1]] = v; }  // surface only (setup)
   }
}

// PA diagonal, one 64-lane workgroup per element, any qdata layout, any (D1D, Q1D) with
// Q1D^2 <= 64: the seven terms of diag(a) = sum_q grad(phi_a)^T O_q grad(phi_a) + m_q phi_a^2
// sum-factorised in three stages through LDS (PADiffusionDiagonal3D / the mass diagonal,
// bilininteg_diffusion_kernels.hpp:369, bilininteg_mass_kernels.hpp:325) -- lanes (qx, qy)
// contract qz, lanes (qx, dz) contract qy, lanes (dy, dz) contract qx and add into the
// L-vector (atomics) or the E-vector.
template <int D, int Q>
__global__ void __launch_bounds__(64)
k_diag_sf(const int *__restrict__ pos, int kind, int ne, const int *__restrict__ gmap,
          const double *__restrict__ qdd, const double *__restrict__ qdm, double *__restrict__ diag, bool out_e,
          const Basis1D *__restrict__ btab)
{
   constexpr int ND = D * D * D, NQ = Q * Q * Q, QQ = Q * Q, DD = D * D, DQ = D * Q;
   static_assert(QQ <= 64, "k_diag_sf needs Q1D <= 8");
   __shared__ double T[7][D][QQ];   // [k][dz][qy qx]
   __shared__ double U[7][DD][Q];   // [k][dz dy][qx]
   const int e = blockIdx.x, t = threadIdx.x;
   if (e >= ne) { return; }
   CBasis *bp = stage_basis(btab);
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
         // terms (11, 22, 33, 12 + 21, 13 + 31, 23 + 32) of the symmetric or general qdata, mass
#pragma unroll
         for (int k = 0; k < 6; k++) { O[k] = qdd ? qd_diag_term(qdd, qdm, pos, kind, NQ, e, k, q) : 0.0; }
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

template <int D, int Q, bool MASS, bool DIFF>
void launch_line_mdq(const ApplyArgs &a, hipStream_t s)
{
   ECM2_VERIFY(a.lelem && a.lelem_off, ERR_INTERNAL, "line kernel needs its element list");
   const int c0 = a.lelem_off[a.blk_begin], c1 = a.lelem_off[a.blk_end];
   if (c1 <= c0) { return; }
   const dim3 grid(c1 - c0), block(64);
#define ECM2_LINE(GG)                                                                                     \
   hipLaunchKernelGGL((k_apply_line<D, Q, MASS, DIFF, GG>), grid, block, 0, s, c0, c1, a.lelem, a.n_owned,   \
                      a.gmap, a.qdd, a.qdm, a.x, a.xg, a.y, a.yg, a.btab, a.part, a.qp)
   if (a.kind == QLAYOUT_AFFINE_E || a.kind == QLAYOUT_TRILINEAR_E)
   {
      if constexpr (DIFF)
      {
         ECM2_VERIFY(a.pw == (MASS ? 2 : 1), ERR_INTERNAL, "compressed point values do not match the integrators");
         if (a.kind == QLAYOUT_AFFINE_E) { ECM2_LINE(1); }
         else { ECM2_LINE(2); }
      }
      else { ECM2_VERIFY(false, ERR_INTERNAL, "compressed qdata needs the diffusion integrator"); }
      return;
   }
   ECM2_LINE(0);
#undef ECM2_LINE
}

template <int D, int Q>
void launch_line_dq(bool mass, bool diff, const ApplyArgs &a, hipStream_t s)
{
   if (mass && diff) { launch_line_mdq<D, Q, true, true>(a, s); }
   else if (mass) { launch_line_mdq<D, Q, true, false>(a, s); }
   else if (diff) { launch_line_mdq<D, Q, false, true>(a, s); }
}

template <int D, int BZ>
void launch_brick(const ApplyArgs &a, hipStream_t s)
{
   constexpr int Q = D + 1;
   const int k0 = a.brick_off[a.blk_begin], k1 = a.brick_off[a.blk_end];
   if (k1 <= k0) { return; }
   ECM2_VERIFY(a.part_brick, ERR_INTERNAL, "brick kernel needs its partial slots");
   const bool split = a.xg || a.yg;
   const int g = a.kind == QLAYOUT_AFFINE_E ? 1 : a.kind == QLAYOUT_TRILINEAR_E ? 2 : 0;
   ECM2_VERIFY(g == 0 || a.pw == 2, ERR_INTERNAL, "bricks need both integrators");
   const dim3 grid(k1 - k0), block(BrickShapeC<D, Q, BZ>::NT);
#define ECM2_BRICK(SP, GG, RG)                                                                             \
   hipLaunchKernelGGL((k_apply_brick_c<D, Q, BZ, SP, GG, RG>), grid, block, 0, s, k0, k1, a.belem, a.bmap,    \
                      a.breg, a.n_owned, a.qdd, a.qdm, a.x, a.xg, a.y, a.yg, a.btab, a.part_brick, a.qp)
#define ECM2_BRICK_G(SP, RG)                    \
   if (g == 1 && a.cdiag) { ECM2_BRICK(SP, 3, RG); } \
   else if (g == 1) { ECM2_BRICK(SP, 1, RG); }  \
   else if (g == 2) { ECM2_BRICK(SP, 2, RG); }  \
   else { ECM2_BRICK(SP, 0, RG); }
   if (split) { ECM2_BRICK_G(true, false) }
   else if (a.breg) { ECM2_BRICK_G(false, true) }
   else { ECM2_BRICK_G(false, false) }
#undef ECM2_BRICK_G
#undef ECM2_BRICK
}

void apply_brick(int D, int Q, const ApplyArgs &a, hipStream_t s)
{
#define ECM2_BRICK_CASE(DD, BZ)                                         \
   if (D == DD && Q == DD + 1 && a.brick_bz == BZ)                      \
   {                                                                    \
      launch_brick<DD, BZ>(a, s);                                       \
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
#undef ECM2_BRICK_CASE
   ECM2_VERIFY(false, ERR_UNSUPPORTED, "no brick kernel for D1D=" << D << " Q1D=" << Q << " bz=" << a.brick_bz);
}

} // namespace

namespace kern
{

bool has_line(int D, int Q)
{
   return (Q == D + 1 || Q == D) && D >= 2 && D <= 7 && Q <= 8;
}

// bricks of 2 x 2 x bz elements for Q1D = D1D + 1 (the default rule), p = 3..6; a
// 2 x 2 x 2 brick's LDS (16 SB doubles) exceeds 160 KiB at p = 6
bool has_brick(int D, int Q, int bz)
{
   if (Q != D + 1 || D < 4 || D > 7) { return false; }
   return bz == 1 || (bz == 2 && D <= 6);
}

int brick_points(int D, int bz) { return (2 * D - 1) * (2 * D - 1) * (bz * (D - 1) + 1); }

void apply_line(int D, int Q, bool mass, bool diff, const ApplyArgs &a, hipStream_t s)
{
   if (a.ne == 0) { return; }
   ECM2_VERIFY(a.btab, ERR_INTERNAL, "line kernel needs the device basis table");
   if (a.brick_bz)
   {
      ECM2_VERIFY(mass && diff, ERR_INTERNAL, "bricks need both integrators");
      apply_brick(D, Q, a, s);
   }
#define ECM2_LINE_CASE(DD, QQ)                                        \
   if (D == DD && Q == QQ)                                            \
   {                                                                  \
      launch_line_dq<DD, QQ>(mass, diff, a, s);                       \
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

// the generic fallback lives in k_misc.hip
void diagonal_generic(const int *pos, int D, int Q, int layout, int ne, const int *gm, const double *qdd,
                      const double *qdm, double *diag, bool out_e, const Basis1D &b, hipStream_t s);

void diagonal(const int *pos, int D, int Q, int layout, int ne, const int *gm, const double *qdd,
              const double *qdm, double *diag, bool out_e, const Basis1D &b, const Basis1D *btab, hipStream_t s)
{
   if (ne == 0) { return; }
#define ECM2_DIAG_CASE(DD, QQ)                                                                             \
   if (D == DD && Q == QQ)                                                                                 \
   {                                                                                                       \
      hipLaunchKernelGGL((k_diag_sf<DD, QQ>), dim3(ne), dim3(64), 0, s, pos, layout, ne, gm, qdd, qdm, diag, \
                         out_e, btab);                                                                     \
      ECM2_HIP(hipGetLastError());                                                                         \
      return;                                                                                              \
   }
   if (btab)
   {
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
      ECM2_DIAG_CASE(2, 4)
      ECM2_DIAG_CASE(3, 5)
      ECM2_DIAG_CASE(4, 6)
      ECM2_DIAG_CASE(5, 7)
      ECM2_DIAG_CASE(6, 8)
   }
#undef ECM2_DIAG_CASE
   diagonal_generic(pos, D, Q, layout, ne, gm, qdd, qdm, diag, out_e, b, s);
}

} // namespace kern
} // namespace ecm2
