// k_tpe.hip -- fused thread-per-element apply and diagonal for p = 1, 2 (gfx950).
//
// One THREAD per element, 64 elements (one 4x4x4 brick) per wave, 4 waves per workgroup.
// Each kernel replaces, in one pass over HBM, ElementRestriction::Mult (restriction.cpp:
// 109-129), the mass and diffusion AddMultPA kernels (bilininteg_mass_kernels.hpp:809-1033,
// bilininteg_diffusion_kernels.hpp:989-1214) and ElementRestriction::MultTranspose
// (restriction.cpp:152-186): gather x into LDS, sum-factorised B/G contractions in
// registers with the qdata streamed once by 1 KiB-per-wave-instruction nontemporal loads,
// then the brick's shared faces assembled in-wave (shuffles) and across the workgroup's
// waves (LDS), and a deterministic store (dofs held once: plain store; shared dofs: dense
// partial slots summed by k_sum_partials in a fixed order).
#include "dev_common.hpp"

namespace ecm2
{
namespace
{
using namespace dev;

// ECM2_SF_W3 (an A/B build): k_apply_tpe_sf (AFFINE / map-addressed blocks, what a
// z-slab rank runs) compiled for three waves per SIMD -- 168 VGPRs, 53,248 B of LDS per workgroup.
#ifndef ECM2_SF_W3
#define ECM2_SF_W3 0
#endif
constexpr bool kSfW3 = ECM2_SF_W3;

// Rows per wave of the LDS region the cross-wave face exchange uses (3 faces of D x D).
template <int D>
struct XwaveRows
{
   static constexpr int ND = D * D * D, R = ND > 3 * D * D ? ND : 3 * D * D;
};

// In-wave assembly of a thread-per-element block's outputs and their store (apply and
// diagonal kernels).  A 4x4x4 brick is one wave: x, y, z neighbours are lanes +1, +4, +16;
// setup-computed lane flags say which faces really coincide (dof-index equality), so any
// element order is correct; bricks make it effective.  SIGNS: apply the map's orientation
// signs before summation (y = A x; the diagonal's signs square away).  Then entries whose
// face was sent away hold nothing; a dof held once in the whole mesh is plain-stored; a
// shared one goes to its dense partial slot [blk][a][lane] (summed in a fixed order by
// k_sum_partials: deterministic, no atomics, no y memset) or, without a partial buffer, is
// atomically added.
// XW: after each direction's in-wave merge, faces shared with another wave of the workgroup
// (lane flags 64|128|256 + the sending wave in bits 9-17, see build_merge_plan) move through
// LDS: the sending lanes (low face, e_dir = 0) park their face in their own wave's region
// xb[w][XR][64] (the kernel's x staging area, no longer read), a barrier, the receiving lanes
// (high face, e_dir = 3) add it.  Every wave of the workgroup must call this (wave_on false:
// barriers only).
// REG (regular blocks, no signs): the lane's dofs are base + X sx + Y sy + Z sz on the block's
// (4(D-1)+1)^3 lattice, shared iff on a block face whose bit is set in mask -- no map reads.
struct TpeReg
{
   int base, sx, sy, sz, mask;
};
// Partial slots: block blk owns part[blk pstride ...]: a regular or lattice-slot block (regf 1 or
// 2) in face-grouped order, [tpe_surface_index(X, Y, Z)] (the summation pass then reads a face's
// two holders as two contiguous runs), any other block as [a][lane].  regf 1 also computes the
// dofs from the lattice (no map reads); regf 2 reads them from the map (dofs not a lattice).
// MAYREG: regf may be nonzero (per block).
// XR: rows per wave of xb (a kernel whose waves stage more than XwaveRows rows passes its stride, so
// a wave's sends land in its own region while the other waves may still read theirs).
template <int D, bool SPLIT, bool SIGNS, bool XW, bool MAYREG = false, int XR = XwaveRows<D>::R, bool XREUSE = false>
__device__ __forceinline__ void tpe_assemble_store(double (&Yo)[D * D * D], const int *__restrict__ mp, int fl,
                                                   int blk, int lane, bool active, int n_owned,
                                                   double *__restrict__ y, double *__restrict__ yg,
                                                   double *__restrict__ part, double *xb, int w, bool wave_on,
                                                   TpeReg rg = {}, int regf = 0, int pstride = D * D * D * 64,
                                                   const int *__restrict__ lm = nullptr)
{
   constexpr int ND = D * D * D;
   // XREUSE: the z faces reuse the x faces' rows (the y merge's barrier orders every wave's x-face
   // reads before any z-face write), so 2 D^2 rows per wave suffice
   static_assert(XR >= (XREUSE ? 2 * D * D : XwaveRows<D>::R), "staging rows");
   auto xrow = [](int dir) { return (XREUSE ? (dir & 1) : dir) * D * D; };
   const bool rr = MAYREG && regf == 1, rs = MAYREG && regf != 0, rl = MAYREG && regf == 2;
   // A lattice-map block's store entries are loaded here, before the face merges: their latency
   // (the map left L2 while the block computed) overlaps the shuffles and barriers instead of
   // preceding the stores.  (An opaque lane offset pins the loads here: hoisted above the
   // compute, 27 live values spill.  Map-addressed blocks keep their loads at the store: the
   // same hoist makes the RM = 0 kernel spill.)
   int lo = 0;
   asm volatile("" : "+v"(lo));
   int gs[ND];
#pragma unroll
   for (int a = 0; a < ND; a++)
   {
      gs[a] = 0;
      if (wave_on && rl)
      {
         const int X = (D - 1) * (lane & 3) + a % D, Y = (D - 1) * ((lane >> 2) & 3) + (a / D) % D,
                   Z = (D - 1) * (lane >> 4) + a / (D * D);
         gs[a] = lm[tpe_lattice_slot(D, X, Y, Z) + lo];
      }
   }
   // (regular and lattice-map blocks carry no orientation signs: checked at setup)
   if (SIGNS && wave_on && !rs)
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
            for (int i = 0; i < D; i++) { xb[((w * XR) + xrow(dir) + j * D + i) * 64 + lane] = Yo[face(0, i, j)]; }
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
                  Yo[face(D - 1, i, j)] += xb[((pw * XR) + xrow(dir) + j * D + i) * 64 + lane - 3 * delta];
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
            int d;
            bool shared;
            constexpr int L = 4 * (D - 1);
            const int X = (D - 1) * (lane & 3) + dx, Y = (D - 1) * ((lane >> 2) & 3) + dy, Z = (D - 1) * (lane >> 4) + dz;
            if (rr)
            {
               d = rg.base + X * rg.sx + Y * rg.sy + Z * rg.sz;
               const int faces = (X == 0) | (X == L) << 1 | (Y == 0) << 2 | (Y == L) << 3 | (Z == 0) << 4 | (Z == L) << 5;
               shared = (faces & rg.mask) != 0;
            }
            else
            {
               const int g = rl ? gs[a] : mp[a * 64];
               d = bdof(g);
               shared = bshared(g);
            }
            double *dst = (!SPLIT || d < n_owned) ? y + d : yg + (d - n_owned);
            if (!shared) { *dst = Yo[a]; }
            else if (part)
            {
               part[(size_t)blk * pstride + (rs ? tpe_surface_index(D, X, Y, Z) : a * 64 + lane)] = Yo[a];
            }
            else { unsafeAtomicAdd(dst, Yo[a]); }
         }
}

// Full per-point qdata (BLOCKED layout), per quadrature row (qy, qz): the 27 gathered dofs
// live in LDS (a private [a][lane] slot per wave: conflict-free ds_read_b64), which frees the
// VGPRs to hold the NEXT row's qdata in flight while the current row is computed (double
// buffering).  Per row: x-values contracted with precomputed B_y B_z, G_y B_z, B_y G_z
// products (scalar loads of the row table), x-forward, weighting by the row's 56-byte points,
// x-transpose, yz-transpose into the element outputs.
template <int D, int Q, bool MASS, bool DIFF, bool SPLIT>
__global__ void __launch_bounds__(256, 1)
k_apply_tpe_pf(int ne, int blk_begin, int blk_end, int n_owned, const int *__restrict__ gmap,
               const double *__restrict__ qdd, const double *__restrict__ qdm,
               const double *__restrict__ x, const double *__restrict__ xg,
               double *__restrict__ y, double *__restrict__ yg, const Basis1D b,
               const double *__restrict__ rowtab, const int *__restrict__ lane_flags,
               double *__restrict__ part)
{
   constexpr int ND = D * D * D, NQ = Q * Q * Q, NQH = (NQ + 1) / 2, DD = D * D;
   constexpr int NR = Q * Q;  // rows
   __shared__ double sX[4][ND][64];
   const int lane = threadIdx.x & 63;
   const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
   const int blk = blk_begin + (int)blockIdx.x * 4 + w;
   if (blk >= blk_end) { return; }  // wave-uniform; no block-wide barrier below
   const int e = blk * 64 + lane;
   const bool active = e < ne;
   const int *mp = gmap + (size_t)blk * ND * 64 + lane;
   double Yo[ND];
#pragma unroll
   for (int a = 0; a < ND; a++) { Yo[a] = 0.0; }

   const double *qd = qdd + (size_t)blk * NQ * 3 * 128 + lane * 2;
   const double *qm = qdm + (size_t)blk * NQH * 128 + lane * 2;
   auto ld2 = [&](const double *p) -> v2d { return __builtin_nontemporal_load(reinterpret_cast<const v2d *>(p)); };
   // row buffers: diffusion pairs (3 per point) and mass values (Q per row)
   v2d cd[Q][3], nd_[Q][3];
   double cm[Q], nm[Q];
   auto load_row = [&](int row, v2d (&dq)[Q][3], double (&mq)[Q]) {
#pragma unroll
      for (int qx = 0; qx < Q; qx++)
      {
         const int q = row * Q + qx;
         if (DIFF)
         {
#pragma unroll
            for (int k = 0; k < 3; k++) { dq[qx][k] = ld2(qd + ((size_t)q * 3 + k) * 128); }
         }
         if (MASS) { mq[qx] = qm[(size_t)(q >> 1) * 128 + (q & 1)]; }
      }
   };
   // the first row's qdata is issued before the gather: its latency overlaps the map -> x chain
   load_row(0, cd, cm);
#pragma unroll
   for (int a = 0; a < ND; a++)
   {
      const int g = mp[a * 64];
      const int d = bdof(g);
      const double v = (!SPLIT || d < n_owned) ? x[d] : xg[d - n_owned];
      sX[w][a][lane] = bneg(g) ? -v : v;
   }

#pragma unroll 1
   for (int row = 0; row < NR; row++)
   {
      if (row + 1 < NR) { load_row(row + 1, nd_, nm); }
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
         if (MASS) { m = cm[qx] * u; }
         if (DIFF)
         {
            // (11,12) (13,22) (23,33)
            const v2d d0 = cd[qx][0], d1 = cd[qx][1], d2 = cd[qx][2];
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
               if (DIFF) { yo += p1 * T1[dx]; yo += p2 * T2[dx]; }
               Yo[(dz * D + dy) * D + dx] = yo;
            }
         }
#pragma unroll
      for (int qx = 0; qx < Q; qx++)
      {
#pragma unroll
         for (int k = 0; k < 3; k++) { cd[qx][k] = nd_[qx][k]; }
         cm[qx] = nm[qx];
      }
   }
   tpe_assemble_store<D, SPLIT, true, false>(Yo, mp, lane_flags[(size_t)blk * 64 + lane], blk, lane, active,
                                             n_owned, y, yg, part, nullptr, w, true);
}

// Thread-per-element apply on AFFINE qdata, sum-factorised per quadrature plane qz: the
// x-values (LDS) are contracted in z once per plane (ZB = B_z X, ZG = G_z X, D^2 each), each of
// the plane's Q rows contracts them in y (3 D^2 multiply-adds instead of the row kernel's
// 3 D^3 on precomputed B_y B_z products), then x / weighting (element matrix C in registers,
// one 16-byte (W beta, W alpha det J) pair per point) / x-transpose; the row's y-transpose
// accumulates into the plane sums SB, SG (2 D^2 + D^2) and the plane ends with one z-transpose
// into the element outputs (2 D^3).  At p = 2 that is 229 FP64 multiply-adds per row.  The
// next row's pairs are in flight while a row computes; in-wave and cross-wave face assembly,
// deterministic store.
// RM: 0 every block map-addressed; 1 every block regular (treg rows, no flag read); 2 per block
// (treg row flag [7], wave-uniform): a regular block's dofs are all owned (checked at setup),
// so it addresses x / y only; 3 every block a lattice-map block (the reference's numbering on a
// Cartesian mesh): the map loads are the first loads of the gather chain.
// TL (TRILINEAR layout, kernels.hpp): the element's trilinear-map coefficients instead of C,
// and the point pair (W beta / det J, W alpha det J); J and adj(J) evaluated at every point: per
// plane (zeta) the J pieces A = c1 + c5 zeta, B = c4 + c7 zeta, Cz = c2 + c6 zeta, per row (eta)
// J[.][0] = A + B eta, G = c3 + c6 eta, H = c5 + c7 eta, per point (xi) J[.][1] = Cz + B xi,
// J[.][2] = G + H xi; then f = (W beta / det J) adj(J) (adj(J)^T grad u), m = (W alpha det J) u --
// PADiffusionSetup3D's D = W beta adj(J) adj(J)^T / det J (bilininteg_diffusion_kernels.cpp:
// 349-362) and the mass setup's W alpha det J, never stored.
// PW: point values per quadrature point (2: the pair; 1: a diffusion-only form's W beta [/ det J]).
template <int D, int Q, bool SPLIT, int RM, bool TL = false, int PW = 2>
__global__ void __launch_bounds__(256, (kSfW3 && !TL) ? 3 : 1)
k_apply_tpe_sf(int ne, int blk_begin, int blk_end, int n_owned, const int *__restrict__ gmap,
               const double *__restrict__ qdd, const double *__restrict__ qdm,
               const double *__restrict__ x, const double *__restrict__ xg,
               double *__restrict__ y, double *__restrict__ yg, const Basis1D b,
               const int *__restrict__ lane_flags, double *__restrict__ part, const int *__restrict__ treg,
               int pstride, const int *__restrict__ lmap, const QPts qp)
{
   constexpr int ND = D * D * D, NQ = Q * Q * Q, NR = Q * Q, WPG = 4;
   // W3 (kSfW3, the three-waves-per-SIMD build): the last x value stays in a register and the face
   // exchange reuses its rows, so three workgroups fit a CU's LDS (26 rows: 159,744 B)
   constexpr bool W3 = kSfW3 && !TL;
   constexpr int XR = W3 ? (ND - 1 > 2 * D * D ? ND - 1 : 2 * D * D) : XwaveRows<D>::R;
   constexpr int XL = W3 ? ND - 1 : ND;  // x values staged in LDS
   __shared__ double sX[WPG][XR][64];  // gathered x; then the cross-wave face exchange
   const int lane = threadIdx.x & 63;
   const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: block data in SGPRs
   double xl = 0.0;                                                  // W3: x value ND - 1
   auto put_x = [&](int a, double v) {
      if (a < XL) { sX[w][a][lane] = v; }
      else { xl = v; }
   };
   // (round-robin dispatch: the XCD-contiguous order of the lattice kernels is 2.6% slower here,
   // profiles/r5/ab_xcd.txt)
   const int blk = blk_begin + (int)blockIdx.x * WPG + w;
   const bool wave_on = blk < blk_end;  // wave-uniform; every wave reaches the store's barriers
   const int e = blk * 64 + lane;
   const bool active = wave_on && e < ne;
   const int *mp = gmap + (size_t)blk * ND * 64 + lane;
   TpeReg rg = {};
   int regf = 0;
   double Yo[ND];
#pragma unroll
   for (int a = 0; a < ND; a++) { Yo[a] = 0.0; }
   if (wave_on)
   {
      // The element matrix and the first rows' pairs are issued first: they do not depend on the
      // gather, so their latency overlaps the (treg ->) (map ->) x chain instead of following it
      // (one memory latency less per wave before the first row computes).
      auto ld2 = [&](const double *p) -> v2d { return __builtin_nontemporal_load(reinterpret_cast<const v2d *>(p)); };
      constexpr int NCE = TL ? kTrilinPairs : 3;
      v2d ce[NCE];
      {
         const double *qc = qdd + (size_t)blk * NCE * 128 + lane * 2;
#pragma unroll
         for (int k = 0; k < NCE; k++) { ce[k] = ld2(qc + k * 128); }
      }
      // TL: coefficient c_{k+1} of coordinate i
      auto cf = [&](int k, int i) -> double {
         const int f = 3 * k + i;
         return (f & 1) ? ce[f >> 1].y : ce[f >> 1].x;
      };
      const double *qa = qdm + (size_t)blk * NQ * 64 * PW + lane * PW;
      v2d ca[Q], na[Q];
      auto load_row = [&](int row, v2d (&aq)[Q]) {
#pragma unroll
         for (int qx = 0; qx < Q; qx++)
         {
            if constexpr (PW == 2) { aq[qx] = ld2(qa + (size_t)(row * Q + qx) * 128); }
            else { aq[qx] = v2d{__builtin_nontemporal_load(qa + (size_t)(row * Q + qx) * 64), 0.0}; }
         }
      };
      // PF2: three row buffers in rotation, each row issues the row two ahead, so 8 KiB per wave
      // are in flight instead of 4 (profiles/r2_ab_pf2.txt: C4 kernel -4.3%); the plane loop is
      // unrolled so the rotation is static.  Map-addressed kernels (RM = 0) keep the ping-pong:
      // unrolled, their register demand exceeds 256 VGPRs; at p = 1 the third buffer costs a wave/SIMD.
      constexpr bool PF2 = RM != 0 && D == 3 && !TL && !W3;  // TL: the runtime plane loop keeps the geometry live once
      v2d ra[PF2 ? 3 : 1][Q];
      if constexpr (PF2)
      {
         load_row(0, ra[0]);
         load_row(1, ra[1]);
      }
      else if constexpr (!W3) { load_row(0, ca); }
      if (RM == 3) { regf = 2; }  // every block lattice-map: no treg row in the gather's chain
      else if (RM)
      {
         const int *r = treg + (size_t)blk * 8;  // wave-uniform: scalar loads
         rg = TpeReg{r[0], r[1], r[2], r[3], r[4]};
         regf = RM == 1 ? 1 : r[7];
      }
      if (regf == 1)
      {
         const int d0 = rg.base + (D - 1) * ((lane & 3) * rg.sx + ((lane >> 2) & 3) * rg.sy + (lane >> 4) * rg.sz);
#pragma unroll
         for (int dz = 0; dz < D; dz++)
#pragma unroll
            for (int dy = 0; dy < D; dy++)
#pragma unroll
               for (int dx = 0; dx < D; dx++)
               {
                  put_x((dz * D + dy) * D + dx, x[d0 + dx * rg.sx + dy * rg.sy + dz * rg.sz]);
               }
      }
      else if (RM >= 2 && regf == 2)
      {
         // lattice-map block: the dofs of the block's lattice points (no signs), each entry a's
         // 64 loads one contiguous sub-block of the map
         const int *lm = lmap + (size_t)blk * tpe_lattice_points(D);
#pragma unroll
         for (int a = 0; a < ND; a++)
         {
            const int X = (D - 1) * (lane & 3) + a % D, Y = (D - 1) * ((lane >> 2) & 3) + (a / D) % D,
                      Z = (D - 1) * (lane >> 4) + a / (D * D);
            const int d = bdof(lm[tpe_lattice_slot(D, X, Y, Z)]);
            put_x(a, (!SPLIT || d < n_owned) ? x[d] : xg[d - n_owned]);
         }
      }
      else
      {
#pragma unroll
         for (int a = 0; a < ND; a++)
         {
            const int g = mp[a * 64];
            const int d = bdof(g);
            const double v = (!SPLIT || d < n_owned) ? x[d] : xg[d - n_owned];
            put_x(a, bneg(g) ? -v : v);
         }
      }
      auto plane = [&](const int qz) {
         double bz[D], gz[D];
#pragma unroll
         for (int dz = 0; dz < D; dz++) { bz[dz] = b.B[qz + MQ * dz]; gz[dz] = b.G[qz + MQ * dz]; }
         double pA[3], pB[3], pC[3];  // TL: the plane's J pieces
         if constexpr (TL)
         {
            const double zt = qp.x[qz];
#pragma unroll
            for (int i = 0; i < 3; i++)
            {
               pA[i] = cf(0, i) + cf(4, i) * zt;
               pB[i] = cf(3, i) + cf(6, i) * zt;
               pC[i] = cf(1, i) + cf(5, i) * zt;
            }
         }
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
                  const int a = (dz * D + dy) * D + dx;
                  const double c = a < XL ? sX[w][a][ll] : xl;
                  zb += bz[dz] * c;
                  zg += gz[dz] * c;
               }
               ZB[dy][dx] = zb; ZG[dy][dx] = zg;
               SB[dy][dx] = 0.0; SG[dy][dx] = 0.0;
            }
         // one row (qz, qy) of Q points: y-forward, x-forward, weighting, x-transpose, y-transpose
         auto row_body = [&](const int qy, const v2d (&cur)[Q]) {
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
            double ja[3], rG[3], rH[3];  // TL: the row's J[.][0] and J[.][2] pieces
            if constexpr (TL)
            {
               const double et = qp.x[qy];
#pragma unroll
               for (int i = 0; i < 3; i++)
               {
                  ja[i] = pA[i] + pB[i] * et;
                  rG[i] = cf(2, i) + cf(5, i) * et;
                  rH[i] = cf(4, i) + cf(6, i) * et;
               }
            }
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
               double m, fx, fy, fz;
               if constexpr (TL)
               {
                  const double xi = qp.x[qx];
                  // J = [ja | jb | jc] (rows: coordinates), adj(J) rows A1., A2., A3.
                  const double jb0 = pC[0] + pB[0] * xi, jb1 = pC[1] + pB[1] * xi, jb2 = pC[2] + pB[2] * xi;
                  const double jc0 = rG[0] + rH[0] * xi, jc1 = rG[1] + rH[1] * xi, jc2 = rG[2] + rH[2] * xi;
                  const double A11 = jb1 * jc2 - jc1 * jb2, A12 = jb2 * jc0 - jb0 * jc2, A13 = jb0 * jc1 - jb1 * jc0;
                  const double A21 = ja[2] * jc1 - ja[1] * jc2, A22 = ja[0] * jc2 - jc0 * ja[2],
                               A23 = ja[1] * jc0 - ja[0] * jc1;
                  const double A31 = ja[1] * jb2 - ja[2] * jb1, A32 = ja[2] * jb0 - ja[0] * jb2,
                               A33 = ja[0] * jb1 - jb0 * ja[1];
                  const double sc = sa.x;  // W beta / det J (setup)
                  double t1 = A11 * ux;
                  t1 += A21 * uy;
                  t1 += A31 * uz;
                  double t2 = A12 * ux;
                  t2 += A22 * uy;
                  t2 += A32 * uz;
                  double t3 = A13 * ux;
                  t3 += A23 * uy;
                  t3 += A33 * uz;
                  m = PW == 2 ? sa.y * u : 0.0;  // W alpha det J
                  fx = sc * (A11 * t1 + A12 * t2 + A13 * t3);
                  fy = sc * (A21 * t1 + A22 * t2 + A23 * t3);
                  fz = sc * (A31 * t1 + A32 * t2 + A33 * t3);
               }
               else
               {
                  m = PW == 2 ? sa.y * u : 0.0;
                  fx = sa.x * (ce[0].x * ux + ce[0].y * uy + ce[1].x * uz);
                  fy = sa.x * (ce[0].y * ux + ce[1].y * uy + ce[2].x * uz);
                  fz = sa.x * (ce[1].x * ux + ce[2].x * uy + ce[2].y * uz);
               }
#pragma unroll
               for (int dx = 0; dx < D; dx++)
               {
                  const double bq = b.B[qx + MQ * dx], gq = b.G[qx + MQ * dx];
                  if (PW == 2) { T0[dx] += bq * m; }
                  T0[dx] += gq * fx;
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
                  if constexpr (W3)
                  {
                     // no plane sums (36 VGPRs): the row's y-transpose goes straight through the
                     // z-transpose into the outputs (54 more FMAs per row)
                     const double pb = by * T0[dx] + gy * T1[dx], pg = by * T2[dx];
#pragma unroll
                     for (int dz = 0; dz < D; dz++) { Yo[(dz * D + dy) * D + dx] += bz[dz] * pb + gz[dz] * pg; }
                  }
                  else
                  {
                     SB[dy][dx] += by * T0[dx];
                     SB[dy][dx] += gy * T1[dx];
                     SG[dy][dx] += by * T2[dx];
                  }
               }
            }
         };
         if constexpr (PF2)
         {
            // the last rows reload the final row (unconditional loads keep the wait counts exact)
#pragma unroll
            for (int qy = 0; qy < Q; qy++)
            {
               const int row = qz * Q + qy;
               __builtin_amdgcn_sched_barrier(0);  // rows stay in program order (no interleaving)
               load_row(row + 2 < NR ? row + 2 : NR - 1, ra[(row + 2) % 3]);
               row_body(qy, ra[row % 3]);
            }
         }
         else if constexpr (W3)
         {
            // one row buffer, no prefetch: the third wave per SIMD hides the row's latency
#pragma unroll
            for (int qy = 0; qy < Q; qy++)
            {
               load_row(qz * Q + qy, ca);
               row_body(qy, ca);
            }
         }
         else if constexpr (Q % 2 == 0)
         {
            // two row buffers in ping-pong, no register moves and no conditional loads: the
            // next row's loads are always the 4 youngest in flight, so a row's data waits on
            // vmcnt(4), never on the row after it (a conditional prefetch plus a buffer copy
            // made the compiler wait for the prefetch itself: one exposed latency per row)
#pragma unroll
            for (int qy = 0; qy < Q; qy += 2)
            {
               const int row = qz * Q + qy;
               load_row(row + 1, na);
               row_body(qy, ca);
               load_row(row + 2 < NR ? row + 2 : NR - 1, ca);  // the next plane's first row (last: a reload)
               row_body(qy + 1, na);
            }
         }
         else
         {
#pragma unroll 1
            for (int qy = 0; qy < Q; qy++)
            {
               const int row = qz * Q + qy;
               if (row + 1 < NR) { load_row(row + 1, na); }
               row_body(qy, ca);
#pragma unroll
               for (int qx = 0; qx < Q; qx++) { ca[qx] = na[qx]; }
            }
         }
#pragma unroll
         for (int dz = 0; dz < D && !W3; dz++)
#pragma unroll
            for (int dy = 0; dy < D; dy++)
#pragma unroll
               for (int dx = 0; dx < D; dx++)
               {
                  Yo[(dz * D + dy) * D + dx] += bz[dz] * SB[dy][dx];
                  Yo[(dz * D + dy) * D + dx] += gz[dz] * SG[dy][dx];
               }
      };
      if constexpr (PF2)
      {
#pragma unroll
         for (int qz = 0; qz < Q; qz++) { plane(qz); }
      }
      else
      {
#pragma unroll 1
         for (int qz = 0; qz < Q; qz++) { plane(qz); }
      }
   }  // wave_on
   tpe_assemble_store<D, SPLIT, RM == 0 || RM == 2, true, RM != 0, XR, W3>(Yo, mp, wave_on ? lane_flags[(size_t)blk * 64 + lane] : 0,
                                                         blk, lane, active, n_owned, y, yg, part, &sX[0][0][0], w,
                                                         wave_on, rg, regf, pstride,
                                                         lmap ? lmap + (size_t)blk * tpe_lattice_points(D) : nullptr);
}

// Lattice coordinates of a block's lattice slots (the inverse of tpe_lattice_slot): X | Y << 5 | Z << 10.
template <int D>
struct LatticeXYZ
{
   static constexpr int L = 4 * (D - 1) + 1, N = L * L * L;
   unsigned short v[N];
   constexpr LatticeXYZ() : v()
   {
      for (int Z = 0; Z < L; Z++)
         for (int Y = 0; Y < L; Y++)
            for (int X = 0; X < L; X++) { v[tpe_lattice_slot(D, X, Y, Z)] = (unsigned short)(X | Y << 5 | Z << 10); }
   }
};
__constant__ LatticeXYZ<3> kLatXYZ3 = LatticeXYZ<3>();  // (the lattice kernel runs at p = 2)
template <int D>
__device__ __forceinline__ unsigned lattice_xyz(int j)
{
   static_assert(D == 3, "p = 2 lattice table");
   return kLatXYZ3.v[j];
}
// The gather's order of the lattice slots: entry p (lane p % 64 of the gather's step p / 64) holds
// lattice slot j | its padded LDS slot << 16.  Within each 64-slot step the slots are dealt into the
// eight 8-lane groups of ds_write_b128 (32 banks: 8 slots of 16 bytes) so that a group's slots differ
// mod 8 as far as the step's residues allow (greedy: the residue with the most slots left first).  In
// slot order the padded rows put two lanes of a group on one bank 63 times per wave (0.35 conflict cycles
// per LDS instruction of the kernel); dealt, 40 (a model of the 27 x 4 reads and 12 writes per wave,
// profiles/r6/lds_model.py -> lds_model.txt).  A step's lanes still read the same map / snapshot lines.
struct LatticeTsGather
{
   static constexpr int N = tpe_lattice_points(3);
   unsigned v[N];
   constexpr LatticeTsGather() : v()
   {
      int lds[N] = {};
      for (int Z = 0; Z < 9; Z++)
         for (int Y = 0; Y < 9; Y++)
            for (int X = 0; X < 9; X++) { lds[tpe_lattice_slot(3, X, Y, Z)] = tsl_slot(X, Y, Z); }
      for (int k0 = 0; k0 < N; k0 += 64)
      {
         const int m = N - k0 < 64 ? N - k0 : 64;
         bool taken[64] = {};
         int out = 0;
         while (out < m)
         {
            const int gsize = m - out < 8 ? m - out : 8;
            bool used[8] = {};
            for (int t = 0; t < gsize; t++)
            {
               int cnt[8] = {};
               for (int i = 0; i < m; i++)
               {
                  if (!taken[i]) { cnt[lds[k0 + i] & 7]++; }
               }
               int best = -1;
               for (int r = 0; r < 8; r++)
               {
                  if (cnt[r] && !used[r] && (best < 0 || cnt[r] > cnt[best])) { best = r; }
               }
               if (best < 0)  // every residue left is in the group already: the largest
               {
                  for (int r = 0; r < 8; r++)
                  {
                     if (cnt[r] && (best < 0 || cnt[r] > cnt[best])) { best = r; }
                  }
               }
               for (int i = 0; i < m; i++)
               {
                  if (!taken[i] && (lds[k0 + i] & 7) == best)
                  {
                     taken[i] = true;
                     v[k0 + out] = (unsigned)(k0 + i) | (unsigned)lds[k0 + i] << 16;
                     out++;
                     break;
                  }
               }
               used[best] = true;
            }
         }
      }
   }
};
constexpr bool ts_gather_is_permutation()
{
   constexpr LatticeTsGather g;
   bool seen[LatticeTsGather::N] = {};
   for (int p = 0; p < LatticeTsGather::N; p++)
   {
      const int j = (int)(g.v[p] & 0xffff);
      if (j >= LatticeTsGather::N || seen[j] || (p / 64) != (j / 64)) { return false; }
      seen[j] = true;
   }
   return true;
}
static_assert(ts_gather_is_permutation(), "the gather order permutes the slots within each 64-slot step");
__constant__ LatticeTsGather kLatTsGather3 = LatticeTsGather();
// The padded LDS slot (tsl_slot, kernels.hpp) of each lattice slot j (regular blocks: slot order).
struct LatticeTsl
{
   static constexpr int N = tpe_lattice_points(3);
   unsigned short v[N];
   constexpr LatticeTsl() : v()
   {
      for (int Z = 0; Z < 9; Z++)
         for (int Y = 0; Y < 9; Y++)
            for (int X = 0; X < 9; X++) { v[tpe_lattice_slot(3, X, Y, Z)] = (unsigned short)tsl_slot(X, Y, Z); }
   }
};
__constant__ LatticeTsl kLatTsl3 = LatticeTsl();

// pairs of the TRILINEAR coefficients (c[3 (k - 1) + i] two per pair) that only the per-plane J
// pieces read: k = 0, 1, 3 -> f = 0..5, 9..11 -> pairs 0, 1, 2, 5 (pair 4 also holds f = 8, a row one)
__device__ __forceinline__ constexpr bool tlb_plane_pair(int k) { return k == 0 || k == 1 || k == 2 || k == 5; }

// TRILINEAR apply for forms whose blocks are all 4x4x4 bricks of one dof lattice (RM 1: regular
// blocks, 3: lattice-map blocks -- the structured numbering and the reference's numbering on a
// brick-tiled mesh), at TWO waves per SIMD.  The per-element kernel above (k_apply_tpe_sf, TL)
// keeps the 27 x-values per element in LDS and the 27 outputs in registers: 408 VGPR+AGPR, one
// wave per SIMD and ~290 AGPR copies per plane, which made it VALU-bound at 0.47 of the HBM peak
// (profiles/r4_*).  Here (a) the block's x values are gathered ONCE per lattice point into LDS in
// the lattice-slot order (729 doubles per 64 elements at p = 2 instead of 1728: the 64 lanes' reads
// of one element entry hit one contiguous sub-block of a residue class, and the gather issues 12
// coalesced map loads per lane instead of 27); (b) the element outputs live in LDS ([a][lane], the
// same region then stages the cross-wave face exchange) and every plane adds its z-transpose into
// them; (c) the per-point pair is (W beta / det J, W alpha det J), so no determinant or division
// per point.  LDS 78.6 KB per workgroup: two workgroups (8 waves) per CU.
template <int D, int Q, bool SPLIT, int RM, int PW = 2>
__global__ void __launch_bounds__(256, 2)
k_apply_tpe_tlb(int ne, int blk_begin, int blk_end, int n_owned, const int *__restrict__ gmap,
                const double *__restrict__ qdd, const double *__restrict__ qdm,
                const double *__restrict__ x, const double *__restrict__ xg,
                double *__restrict__ y, double *__restrict__ yg, const Basis1D b,
                const int *__restrict__ lane_flags, double *__restrict__ part,
                const int *__restrict__ treg, int pstride, const int *__restrict__ lmap, const QPts qp)
{
   static_assert(RM == 1 || RM == 3, "lattice blocks only");
   static_assert(Q % 2 == 0, "ping-pong rows");
   constexpr int ND = D * D * D, NQ = Q * Q * Q, NR = Q * Q, XR = XwaveRows<D>::R, WPG = 4, P = D - 1;
   constexpr int NLP = tpe_lattice_points(D);
   static_assert(XR >= ND, "outputs fit the staging rows");
   __shared__ double sXL[WPG][NLP];   // the block's x values in lattice-slot order
   __shared__ double sY[WPG][XR][64]; // element outputs [a][lane]; then the cross-wave face exchange
   const int lane = threadIdx.x & 63;
   const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
   const int blk = blk_begin + xcd_contiguous((int)blockIdx.x, (int)gridDim.x) * WPG + w;  // (as k_apply_tpe_ts)
   const bool wave_on = blk < blk_end;  // wave-uniform; every wave reaches the barriers
   const int e = blk * 64 + lane;
   const bool active = wave_on && e < ne;
   const int *mp = gmap + (size_t)blk * ND * 64 + lane;
   const int ex = lane & 3, ey = (lane >> 2) & 3, ez = lane >> 4;
   TpeReg rg = {};
   const int regf = RM == 1 ? 1 : 2;
   auto ld2 = [&](const double *p) -> v2d { return __builtin_nontemporal_load(reinterpret_cast<const v2d *>(p)); };
   constexpr int NCE = kTrilinPairs;
   v2d ce[NCE];
   const double *qa = qdm + (size_t)blk * NQ * 64 * PW + lane * PW;
   auto ldp = [&](int q) -> v2d {  // the point values of point q (PW = 1: W beta / det J alone)
      if constexpr (PW == 2) { return ld2(qa + (size_t)q * 128); }
      else { return v2d{__builtin_nontemporal_load(qa + (size_t)q * 64), 0.0}; }
   };
   v2d ca[Q];  // point values of the row in flight
   auto load_row = [&](int row, v2d (&aq)[Q]) {
#pragma unroll
      for (int qx = 0; qx < Q; qx++) { aq[qx] = ldp(row * Q + qx); }
   };
   if (wave_on)
   {
      // geometry and the first row's pairs first: independent of the gather chain
      const double *qc = qdd + (size_t)blk * NCE * 128 + lane * 2;
#pragma unroll
      for (int k = 0; k < NCE; k++)
      {
         if (!tlb_plane_pair(k)) { ce[k] = ld2(qc + k * 128); }  // (the plane-only pairs: per plane)
      }
      load_row(0, ca);
      if (RM == 1)
      {
         const int *r = treg + (size_t)blk * 8;  // wave-uniform: scalar loads
         rg = TpeReg{r[0], r[1], r[2], r[3], r[4]};
      }
      const int *lm = lmap + (size_t)blk * NLP;
#pragma unroll
      for (int k = 0; k < (NLP + 63) / 64; k++)
      {
         const int j = lane + 64 * k;
         if (j < NLP)
         {
            int d;
            if (RM == 3) { d = bdof(lm[j]); }
            else
            {
               const unsigned v = lattice_xyz<D>(j);
               d = rg.base + (int)(v & 31) * rg.sx + (int)((v >> 5) & 31) * rg.sy + (int)(v >> 10) * rg.sz;
            }
            sXL[w][j] = (!SPLIT || d < n_owned) ? x[d] : xg[d - n_owned];
         }
      }
#pragma unroll
      for (int a = 0; a < ND; a++) { sY[w][a][lane] = 0.0; }
   }
   __syncthreads();  // the lattice is read by every lane of the wave
   if (wave_on)
   {
      auto cf = [&](int k, int i) -> double {
         const int f = 3 * k + i;
         return (f & 1) ? ce[f >> 1].y : ce[f >> 1].x;
      };
      // lane part of a lattice slot per residue class (cx, cy): ((ez) ny + ey) nx + ex
      auto lane_base = [&](int cx, int cy) {
         const int nx = tpe_lattice_class_n(cx), ny = tpe_lattice_class_n(cy);
         return (ez * ny + ey) * nx + ex;
      };
#pragma unroll 1
      for (int qz = 0; qz < Q; qz++)
      {
         double bz[D], gz[D];
#pragma unroll
         for (int dz = 0; dz < D; dz++) { bz[dz] = b.B[qz + MQ * dz]; gz[dz] = b.G[qz + MQ * dz]; }
         double pA[3], pB[3], pC[3];  // the plane's J pieces
         {
            {
               // the coefficients only the plane pieces use (c1, c2, c4) are read again per plane (an
               // L2 hit) instead of being held through the rows: 16 VGPRs, which removes the 11-14
               // spilled values (profiles/r4/ab_tlr.txt: kernel -2.7% trilinear, -3.4% drop-in).  (The
               // opaque pointer keeps the loads in the plane loop.)
               const double *qcp = qdd + (size_t)blk * NCE * 128 + lane * 2;
               asm volatile("" : "+v"(qcp));
#pragma unroll
               for (int k = 0; k < NCE; k++)
               {
                  if (tlb_plane_pair(k)) { ce[k] = *reinterpret_cast<const v2d *>(qcp + k * 128); }
               }
            }
            // opaque per plane: otherwise the compiler hoists every plane's and row's J pieces out of
            // the plane loop into a table (in scratch)
            double zt = qp.x[qz];
            asm volatile("" : "+s"(zt));
#pragma unroll
            for (int i = 0; i < 3; i++)
            {
               pA[i] = cf(0, i) + cf(4, i) * zt;
               pB[i] = cf(3, i) + cf(6, i) * zt;
               pC[i] = cf(1, i) + cf(5, i) * zt;
            }
         }
         // the plane's z-forward partials from the lattice (ZB = B_z X, ZG = G_z X): 36 VGPRs that
         // spill 2 values per plane into scratch, against 81 instead of 27 multiply-adds per row
         // when every row re-reads the lattice (profiles/r4/ab_tlz_pf2.txt: kernel -2..-3%)
         double SB[D][D], SG[D][D], ZB[D][D], ZG[D][D];
#pragma unroll
         for (int dy = 0; dy < D; dy++)
#pragma unroll
            for (int dx = 0; dx < D; dx++)
            {
               SB[dy][dx] = 0.0; SG[dy][dx] = 0.0;
               int lb = lane_base(dx % P, dy % P);
               asm volatile("" : "+v"(lb));
               double zb = 0.0, zg = 0.0;
#pragma unroll
               for (int dz = 0; dz < D; dz++)
               {
                  const int cx = dx % P, cy = dy % P, cz = dz % P;
                  const int nx = tpe_lattice_class_n(cx), ny = tpe_lattice_class_n(cy);
                  const int sl = tpe_lattice_class_off(D, cx, cy, cz) + ((dz / P) * ny + dy / P) * nx + dx / P;
                  const double c = sXL[w][lb + sl];
                  zb += bz[dz] * c;
                  zg += gz[dz] * c;
               }
               ZB[dy][dx] = zb; ZG[dy][dx] = zg;
            }
         auto row_body = [&](const int qy, v2d (&cur)[Q], const int next_row) {
            double Y00[D], Y01[D], Y10[D];
#pragma unroll
            for (int dx = 0; dx < D; dx++)
            {
               double u = 0.0, v = 0.0, wv = 0.0;
#pragma unroll
               for (int dy = 0; dy < D; dy++)
               {
                  const double by = b.B[qy + MQ * dy], gy = b.G[qy + MQ * dy];
                  const double zb = ZB[dy][dx], zg = ZG[dy][dx];
                  u += by * zb;
                  v += gy * zb;
                  wv += by * zg;
               }
               Y00[dx] = u; Y01[dx] = v; Y10[dx] = wv;
            }
            double T0[D], T1[D], T2[D];
#pragma unroll
            for (int dx = 0; dx < D; dx++) { T0[dx] = 0.0; T1[dx] = 0.0; T2[dx] = 0.0; }
            double ja[3], rG[3], rH[3];  // the row's J[.][0] and J[.][2] pieces
            {
               double et = qp.x[qy];
               asm volatile("" : "+s"(et));  // (as zt: the rows' pieces stay in the loop)
#pragma unroll
               for (int i = 0; i < 3; i++)
               {
                  ja[i] = pA[i] + pB[i] * et;
                  rG[i] = cf(2, i) + cf(5, i) * et;
                  rH[i] = cf(4, i) + cf(6, i) * et;
               }
            }
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
               // the next row's pair of this point goes into the slot just read: one row in flight
               // (two rows, in two buffers: +3% kernel time, profiles/r4/ab_pfd.txt)
               cur[qx] = ldp(next_row * Q + qx);
               const double xi = qp.x[qx];
               // J = [ja | jb | jc] (rows: coordinates), adj(J) rows A1., A2., A3.
               const double jb0 = pC[0] + pB[0] * xi, jb1 = pC[1] + pB[1] * xi, jb2 = pC[2] + pB[2] * xi;
               const double jc0 = rG[0] + rH[0] * xi, jc1 = rG[1] + rH[1] * xi, jc2 = rG[2] + rH[2] * xi;
               const double A11 = jb1 * jc2 - jc1 * jb2, A12 = jb2 * jc0 - jb0 * jc2, A13 = jb0 * jc1 - jb1 * jc0;
               const double A21 = ja[2] * jc1 - ja[1] * jc2, A22 = ja[0] * jc2 - jc0 * ja[2],
                            A23 = ja[1] * jc0 - ja[0] * jc1;
               const double A31 = ja[1] * jb2 - ja[2] * jb1, A32 = ja[2] * jb0 - ja[0] * jb2,
                            A33 = ja[0] * jb1 - jb0 * ja[1];
               // t = (W beta / det J) adj(J)^T grad u, f = adj(J) t, m = (W alpha det J) u
               const double sux = sa.x * ux, suy = sa.x * uy, suz = sa.x * uz;
               double t1 = A11 * sux;
               t1 += A21 * suy;
               t1 += A31 * suz;
               double t2 = A12 * sux;
               t2 += A22 * suy;
               t2 += A32 * suz;
               double t3 = A13 * sux;
               t3 += A23 * suy;
               t3 += A33 * suz;
               const double m = PW == 2 ? sa.y * u : 0.0;
               double fx = A11 * t1;
               fx += A12 * t2;
               fx += A13 * t3;
               double fy = A21 * t1;
               fy += A22 * t2;
               fy += A23 * t3;
               double fz = A31 * t1;
               fz += A32 * t2;
               fz += A33 * t3;
#pragma unroll
               for (int dx = 0; dx < D; dx++)
               {
                  const double bq = b.B[qx + MQ * dx], gq = b.G[qx + MQ * dx];
                  if (PW == 2) { T0[dx] += bq * m; }
                  T0[dx] += gq * fx;
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
                  SB[dy][dx] += by * T0[dx];
                  SB[dy][dx] += gy * T1[dx];
                  SG[dy][dx] += by * T2[dx];
               }
            }
         };
#pragma unroll
         for (int qy = 0; qy < Q; qy++)
         {
            const int row = qz * Q + qy;
            __builtin_amdgcn_sched_barrier(0);  // rows stay in program order (no interleaved live ranges)
            row_body(qy, ca, row + 1 < NR ? row + 1 : NR - 1);  // (the last row reloads itself: exact wait counts)
         }
         // the plane's z-transpose into the outputs (private [a][lane] slots: same-lane RMW)
#pragma unroll
         for (int dz = 0; dz < D; dz++)
#pragma unroll
            for (int dy = 0; dy < D; dy++)
#pragma unroll
               for (int dx = 0; dx < D; dx++)
               {
                  double &yo = sY[w][(dz * D + dy) * D + dx][lane];
                  double v = yo;
                  v += bz[dz] * SB[dy][dx];
                  v += gz[dz] * SG[dy][dx];
                  yo = v;
               }
      }
   }  // wave_on
   double Yo[ND];
#pragma unroll
   for (int a = 0; a < ND; a++) { Yo[a] = wave_on ? sY[w][a][lane] : 0.0; }
   tpe_assemble_store<D, SPLIT, false, true, true>(Yo, mp, wave_on ? lane_flags[(size_t)blk * 64 + lane] : 0, blk, lane,
                                                  active, n_owned, y, yg, part, &sY[0][0][0], w, wave_on, rg, regf,
                                                  pstride, lmap ? lmap + (size_t)blk * NLP : nullptr);
}

// AFFINE apply with the diffusion coefficient evaluated from a snapshot of its temperature field
// (TS: ApplyArgs::tsnap).  In the bioheat form beta = k(T) is a law of T, an H1 grid function on the
// form's own space (GridFunctionCoefficient, coefficient.cpp:250-253, possibly composed with a law as
// TransformedCoefficient::Eval does, coefficient.cpp:262): the reference evaluates it at the
// quadrature points at Assemble (CoefficientVector::Project, coefficient.cpp:2052-2070, then
// PADiffusionSetup3D stores W beta adj(J) adj(J)^T / det J).  Here Assemble keeps a snapshot of the
// field at its dofs and the kernel interpolates it at the points in the same sum factorisation as u
// (per plane 27, per row 9, per point 3 multiply-adds), so no W beta is streamed:
// * LAW = false: the snapshot is T' = A + B T (an affine or identity law applied to the dofs: the
//   basis sums to one, so the interpolated T' is the law at the point) and the weight-scaled basis
//   w_q B (bw) gives W_q beta(x_q) directly;
// * LAW = true: the snapshot is T itself, interpolated with B (bw = b) to T(x_q), where the laws are
//   applied (law_d: any grid-function law, e.g. the perfusion law; law_m: a mass law of the same
//   field) and multiplied by W_q = w_qx w_qy w_qz.
// MM: the mass -- 0 none; 1 W alpha det J streamed per point; 2 one stored value per element,
// (c alpha) det J (a constant coefficient folded in, or the mass law evaluated here), times W_q: no
// per-point stream at all.  x and T' are gathered once per lattice point (the block's 729 lattice
// slots, as k_apply_tpe_tlb) into one LDS region that the cross-wave face exchange reuses afterwards.
// Lattice blocks only (RM 1 regular, 3 lattice-map), p = 2.
template <int D, int Q, bool SPLIT, int RM, int MM, bool LAW, bool CD>
__global__ void __launch_bounds__(256, 2)
k_apply_tpe_ts(int ne, int blk_begin, int blk_end, int n_owned, const int *__restrict__ gmap,
               const double *__restrict__ qdd, const double *__restrict__ qdm,
               const double *__restrict__ x, const double *__restrict__ xg, const double *__restrict__ tsn,
               double *__restrict__ y, double *__restrict__ yg, const Basis1D b, const Basis1D bw,
               const int *__restrict__ lane_flags, double *__restrict__ part, const int *__restrict__ treg,
               int pstride, const int *__restrict__ lmap, const QPts qw, const PointLaw law_d, const PointLaw law_m,
               double *__restrict__ en)
{
   static_assert(RM == 1 || RM == 3, "lattice blocks only");
   static_assert(D == 3 && Q == 4, "p = 2");
   constexpr bool MASS = MM != 0;
   constexpr int ND = D * D * D, NR = Q * Q, XR = XwaveRows<D>::R, WPG = 4, P = D - 1;
   constexpr int NLP = tpe_lattice_points(D);
   // rows per wave: the padded (x, T') image (tsl_points pairs, conflict-free 16-byte reads), which
   // the cross-wave face exchange (XR rows) reuses
   constexpr int XRS = (2 * tsl_points() + 63) / 64 > XR ? (2 * tsl_points() + 63) / 64 : XR;
   __shared__ double sU[WPG][XRS][64];  // per wave: (x, T') lattice pairs; then the cross-wave face exchange
   const int lane = threadIdx.x & 63;
   const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
   // XCD-contiguous workgroup order: consecutive (Morton-adjacent) brick groups share one XCD's L2
   // for the x / T' lattice faces they both gather (kernel -1.5..-2.3%, profiles/r5/ab_xcd.txt)
   const int blk = blk_begin + xcd_contiguous((int)blockIdx.x, (int)gridDim.x) * WPG + w;
   const bool wave_on = blk < blk_end;  // wave-uniform; every wave reaches the barriers
   const int e = blk * 64 + lane;
   const bool active = wave_on && e < ne;
   const int *mp = gmap + (size_t)blk * ND * 64 + lane;
   const int ex = lane & 3, ey = (lane >> 2) & 3, ez = lane >> 4;
   // (x, T') pairs per lattice slot: one 16-byte LDS read per point (two 8-byte arrays: +3.5% kernel
   // time, profiles/r4/ab_pfd.txt)
   v2d *sPL = reinterpret_cast<v2d *>(&sU[w][0][0]);
   TpeReg rg = {};
   const int regf = RM == 1 ? 1 : 2;
   double Yo[ND];
#pragma unroll
   for (int a = 0; a < ND; a++) { Yo[a] = 0.0; }
   auto ld2 = [&](const double *p) -> v2d { return __builtin_nontemporal_load(reinterpret_cast<const v2d *>(p)); };
   v2d ce[3];
   const double *qa = qdm + (size_t)blk * NR * Q * 64 + lane;  // MM 1: W alpha det J, [blk][q][lane]
   // three row buffers in rotation, each row issues the row two ahead (the plane loop is unrolled)
   double ra[3][Q];
   auto load_row = [&](int row, double (&aq)[Q]) {
#pragma unroll
      for (int qx = 0; qx < Q; qx++) { aq[qx] = MM == 1 ? __builtin_nontemporal_load(qa + (size_t)(row * Q + qx) * 64) : 0.0; }
   };
   double mel = 0.0;  // MM 2: the element's (c alpha) det J, [blk][lane]
   if (wave_on)
   {
      const double *qc = qdd + (size_t)blk * 3 * 128 + lane * 2;
#pragma unroll
      for (int k = 0; k < 3; k++) { ce[k] = ld2(qc + k * 128); }
      load_row(0, ra[0]);
      load_row(1, ra[1]);
      if (MM == 2) { mel = qdm[(size_t)blk * 64 + lane]; }
      if (RM == 1)
      {
         const int *r = treg + (size_t)blk * 8;  // wave-uniform: scalar loads
         rg = TpeReg{r[0], r[1], r[2], r[3], r[4]};
      }
      const int *lm = lmap + (size_t)blk * NLP;
#pragma unroll
      for (int k = 0; k < (NLP + 63) / 64; k++)
      {
         const int p = lane + 64 * k;
         if (p < NLP)
         {
            // lattice-map blocks: the slots dealt for the writes' banks (the lanes of a step still read the
            // same map and snapshot lines); regular blocks: slot order (j = p), whose x / T' gathers of a
            // step stay on few lines -- dealt, they cost the structured Mult 3% (profiles/r6/ab_gather.txt)
            int j, ls;
            if (RM == 3)
            {
               const unsigned g = kLatTsGather3.v[p];
               j = (int)(g & 0xffff);
               ls = (int)(g >> 16);
            }
            else
            {
               j = p;
               ls = kLatTsl3.v[p];
            }
            int d;
            if (RM == 3) { d = bdof(lm[j]); }
            else
            {
               const unsigned v = lattice_xyz<D>(j);
               d = rg.base + (int)(v & 31) * rg.sx + (int)((v >> 5) & 31) * rg.sy + (int)(v >> 10) * rg.sz;
            }
            // (lattice-map blocks: the snapshot is stored in their slot order, a contiguous read)
            sPL[ls] = v2d{(!SPLIT || d < n_owned) ? x[d] : xg[d - n_owned], RM == 3 ? tsn[(size_t)blk * NLP + j] : tsn[d]};
         }
      }
   }
   __syncthreads();  // the lattices are read by every lane of the wave
   if (wave_on)
   {
      auto lane_base = [&](int cx, int cy) {  // (the padded image: tsl_slot)
         const int nx = tpe_lattice_class_n(cx), ny = tpe_lattice_class_n(cy);
         return ez * tsl_sz(nx, ny) + ey * tsl_sy(nx) + ex;
      };
      auto plane = [&](const int qz) {
         double bz[D], gz[D], wz[D];
#pragma unroll
         for (int dz = 0; dz < D; dz++)
         {
            bz[dz] = b.B[qz + MQ * dz]; gz[dz] = b.G[qz + MQ * dz]; wz[dz] = LAW ? bz[dz] : bw.B[qz + MQ * dz];
         }
         double ZB[D][D], ZG[D][D], ZT[D][D], SB[D][D], SG[D][D];
#pragma unroll
         for (int dy = 0; dy < D; dy++)
#pragma unroll
            for (int dx = 0; dx < D; dx++)
            {
               int lb = lane_base(dx % P, dy % P);
               asm volatile("" : "+v"(lb));  // the plane re-reads the lattices (no 54 live values)
               double zb = 0.0, zg = 0.0, zt = 0.0;
#pragma unroll
               for (int dz = 0; dz < D; dz++)
               {
                  const int cx = dx % P, cy = dy % P, cz = dz % P;
                  const int nx = tpe_lattice_class_n(cx), ny = tpe_lattice_class_n(cy);
                  const int sl = tsl_class_off(cx, cy, cz) + (dz / P) * tsl_sz(nx, ny) + (dy / P) * tsl_sy(nx) + dx / P;
                  const v2d ct = sPL[lb + sl];
                  const double c = ct.x, t = ct.y;
                  zb += bz[dz] * c;
                  zg += gz[dz] * c;
                  zt += wz[dz] * t;
               }
               ZB[dy][dx] = zb; ZG[dy][dx] = zg; ZT[dy][dx] = zt;
               SB[dy][dx] = 0.0; SG[dy][dx] = 0.0;
            }
         auto row_body = [&](const int qy, const double (&cur)[Q]) {
            double Y00[D], Y01[D], Y10[D], YT[D];
            const double wyz = qw.x[qy] * qw.x[qz];  // (LAW or MM 2: W_q = w_qx w_qy w_qz)
#pragma unroll
            for (int dx = 0; dx < D; dx++)
            {
               double u = 0.0, v = 0.0, wv = 0.0, t = 0.0;
#pragma unroll
               for (int dy = 0; dy < D; dy++)
               {
                  const double by = b.B[qy + MQ * dy], gy = b.G[qy + MQ * dy];
                  const double wy = LAW ? by : bw.B[qy + MQ * dy];
                  u += by * ZB[dy][dx];
                  v += gy * ZB[dy][dx];
                  wv += by * ZG[dy][dx];
                  t += wy * ZT[dy][dx];
               }
               Y00[dx] = u; Y01[dx] = v; Y10[dx] = wv; YT[dx] = t;
            }
            double T0[D], T1[D], T2[D];
#pragma unroll
            for (int dx = 0; dx < D; dx++) { T0[dx] = 0.0; T1[dx] = 0.0; T2[dx] = 0.0; }
#pragma unroll
            for (int qx = 0; qx < Q; qx++)
            {
               double u = 0.0, ux = 0.0, uy = 0.0, uz = 0.0, wb = 0.0;
#pragma unroll
               for (int dx = 0; dx < D; dx++)
               {
                  const double bq = b.B[qx + MQ * dx], gq = b.G[qx + MQ * dx];
                  const double wq = LAW ? bq : bw.B[qx + MQ * dx];
                  u += bq * Y00[dx];
                  ux += gq * Y00[dx];
                  uy += bq * Y01[dx];
                  uz += bq * Y10[dx];
                  wb += wq * YT[dx];  // LAW: T(x_q), else W_q beta(x_q)
               }
               double mc = 0.0;  // W alpha det J
               if (LAW || MM == 2)
               {
                  const double Wq = wyz * qw.x[qx];
                  if (MM == 2) { mc = Wq * mel; }
                  if (LAW)
                  {
                     const double tq = wb;
                     wb = Wq * point_law(law_d, tq);
                     if (MM == 2) { mc *= point_law(law_m, tq); }
                  }
               }
               if (MM == 1) { mc = cur[qx]; }
               const double m = MASS ? mc * u : 0.0;  // W alpha det J u
               double fx, fy, fz;
               if constexpr (CD)
               {
                  // axis-aligned elements (C diagonal, checked at setup): the same values as the general
                  // product below, whose off-diagonal terms then add exact zeros
                  fx = ce[0].x * ux; fy = ce[1].y * uy; fz = ce[2].y * uz;
               }
               else
               {
                  fx = ce[0].x * ux; fy = ce[0].y * ux; fz = ce[1].x * ux;
                  fx += ce[0].y * uy; fy += ce[1].y * uy; fz += ce[2].x * uy;
                  fx += ce[1].x * uz; fy += ce[2].x * uz; fz += ce[2].y * uz;
               }
               fx *= wb; fy *= wb; fz *= wb;
#pragma unroll
               for (int dx = 0; dx < D; dx++)
               {
                  const double bq = b.B[qx + MQ * dx], gq = b.G[qx + MQ * dx];
                  if (MASS) { T0[dx] += bq * m; }
                  T0[dx] += gq * fx;
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
                  SB[dy][dx] += by * T0[dx];
                  SB[dy][dx] += gy * T1[dx];
                  SG[dy][dx] += by * T2[dx];
               }
            }
         };
#pragma unroll
         for (int qy = 0; qy < Q; qy++)
         {
            const int row = qz * Q + qy;
            __builtin_amdgcn_sched_barrier(0);  // rows stay in program order (no interleaving)
            load_row(row + 2 < NR ? row + 2 : NR - 1, ra[(row + 2) % 3]);  // (the last rows reload the final row)
            row_body(qy, ra[row % 3]);
         }
#pragma unroll
         for (int dz = 0; dz < D; dz++)
#pragma unroll
            for (int dy = 0; dy < D; dy++)
#pragma unroll
               for (int dx = 0; dx < D; dx++)
               {
                  Yo[(dz * D + dy) * D + dx] += bz[dz] * SB[dy][dx];
                  Yo[(dz * D + dy) * D + dx] += gz[dz] * SG[dy][dx];
               }
      };
#pragma unroll
      for (int qz = 0; qz < Q; qz++) { plane(qz); }
   }  // wave_on
   if (en)  // (uniform) the Mult's energy x^T A x = sum_e X_e . (A_e X_e), one partial per workgroup
   {
      // CGSolver's den = (A d, d) (solvers.cpp:993) without a dot pass: the element outputs are
      // complete here and X_e is still in the lattice image (ConstrainedOperator's zeroed ess entries
      // included); PAForm::mult_energy documents the ess correction.  Fixed order: lanes, then waves.
      __shared__ double red[WPG];
      double e_l = 0.0;
      if (wave_on && active)
      {
#pragma unroll
         for (int dz = 0; dz < D; dz++)
#pragma unroll
            for (int dy = 0; dy < D; dy++)
#pragma unroll
               for (int dx = 0; dx < D; dx++)
               {
                  const double xv = sPL[tsl_slot(2 * ex + dx, 2 * ey + dy, 2 * ez + dz)].x;
                  e_l += xv * Yo[(dz * D + dy) * D + dx];
               }
      }
      for (int off = 32; off > 0; off >>= 1) { e_l += __shfl_down(e_l, off, 64); }
      if (lane == 0) { red[w] = e_l; }
      __syncthreads();
      if (threadIdx.x == 0) { en[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]); }
   }
   tpe_assemble_store<D, SPLIT, false, true, true, XRS>(Yo, mp, wave_on ? lane_flags[(size_t)blk * 64 + lane] : 0, blk, lane,
                                                       active, n_owned, y, yg, part, &sU[0][0][0], w, wave_on, rg, regf,
                                                       pstride, lmap ? lmap + (size_t)blk * NLP : nullptr);
}

// Latency variant of k_apply_tpe_sf for small block ranges (the boundary elements of the
// overlapped distributed-Mult schedule, behind the exchange): one workgroup per 64-element block, its
// four waves gather the x-values together and take one quadrature plane each (all of the
// plane's pairs loaded up front), so a block costs one plane's latency instead of four.
// Waves 1..3 hand their partial outputs to wave 0 through LDS, which adds them in a fixed
// order (deterministic) and assembles / stores exactly like k_apply_tpe_sf (in-wave only).
template <int D, int Q, bool SPLIT>
__global__ void __launch_bounds__(256)
k_apply_tpe_pp(int ne, int blk_begin, int n_owned, const int *__restrict__ gmap,
               const double *__restrict__ qdd, const double *__restrict__ qdm,
               const double *__restrict__ x, const double *__restrict__ xg,
               double *__restrict__ y, double *__restrict__ yg, const Basis1D b,
               const int *__restrict__ lane_flags, double *__restrict__ part, int pstride)
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
               T0[dx] += bq * m;
               T0[dx] += gq * fx;
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
               SB[dy][dx] += by * T0[dx];
               SB[dy][dx] += gy * T1[dx];
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
                                             n_owned, y, yg, part, nullptr, 0, true, TpeReg{}, 0, pstride);
}

// PA diagonal, thread per element on the blocked layout (PADiffusionDiagonal3D and the
// mass diagonal, bilininteg_diffusion_kernels.hpp:369, bilininteg_mass_kernels.hpp:325,
// assembled like AssembleDiagonal's E->L transpose, bilinearform_ext.cpp:370-454):
//   diag(a) = sum_q grad(phi_a)^T O_q grad(phi_a) + m_q phi_a^2,  phi_a = B_x B_y B_z,
// sum-factorised per quadrature row (qy, qz): seven x-contractions S_k(dx) of the row's
// qdata, then the (dy, dz) factors of the row from a table, [6][dz][dy] = (By Bz)^2,
// (Gy Bz)^2, (By Gz)^2, Gy By Bz^2, By^2 Gz Bz, Gy By Gz Bz.  Output assembled and stored
// exactly like the apply kernels' (in-wave faces, cross-wave faces on AFFINE, plain stores,
// partial slots): every diagonal entry written once, deterministic, no memset.
template <int D, int Q, bool MASS, bool DIFF, bool SPLIT, bool AFF, bool XWV = AFF>
__global__ void __launch_bounds__(256)
k_diag_tpe(int ne, int blk_begin, int blk_end, int n_owned, const int *__restrict__ gmap,
           const double *__restrict__ qdd, const double *__restrict__ qdm, double *__restrict__ y,
           double *__restrict__ yg, const Basis1D b, const double *__restrict__ drow,
           const int *__restrict__ lane_flags, double *__restrict__ part, const int *__restrict__ treg, int pstride,
           const int *__restrict__ lmap)
{
   constexpr int ND = D * D * D, NQ = Q * Q * Q, NQH = (NQ + 1) / 2, DD = D * D, XR = XwaveRows<D>::R, WPG = 4;
   // XWV: cross-wave face exchange, as the apply's plan (AFFINE; TRILINEAR forms, whose diagonal
   // reads their full per-point qdata: AFF false, XWV true)
   __shared__ double xb[XWV ? WPG * XR * 64 : 1];
   const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
   const int blk = blk_begin + blockIdx.x * WPG + w;
   const bool wave_on = blk < blk_end;  // wave-uniform
   if (!XWV && !wave_on) { return; }    // no block-wide barrier without the exchange
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
   // regular blocks (treg row flag): the apply's face-grouped partial slots
   TpeReg rg = {};
   int regf = 0;
   if (treg && wave_on)
   {
      const int *r = treg + (size_t)blk * 8;
      rg = TpeReg{r[0], r[1], r[2], r[3], r[4]};
      regf = r[7];
   }
   tpe_assemble_store<D, SPLIT, false, XWV, true>(Yo, mp, wave_on ? lane_flags[(size_t)blk * 64 + lane] : 0, blk,
                                                  lane, active, n_owned, y, yg, part, xb, w, wave_on, rg, regf,
                                                  pstride, lmap ? lmap + (size_t)blk * tpe_lattice_points(D) : nullptr);
}

template <int D, int Q, bool MASS, bool DIFF, bool SPLIT>
void launch_tpe(const ApplyArgs &a, const Basis1D &b, const double *rowtab, hipStream_t s)
{
   const int nb = a.blk_end - a.blk_begin;
   const dim3 grid((nb + 3) / 4), block(256);
   // compressed layouts: both integrators (PW 2) or a diffusion-only form (PW 1)
   constexpr int PW = MASS ? 2 : 1;
   if (a.kind == QLAYOUT_TRILINEAR)
   {
      if constexpr (DIFF)
      {
         ECM2_VERIFY(a.pw == PW, ERR_INTERNAL, "TRILINEAR point values do not match the integrators");
#define ECM2_TL(KT)                                                                                           \
   hipLaunchKernelGGL(KT, grid, block, 0, s, a.ne, a.blk_begin, a.blk_end, a.n_owned, a.gmap, a.qdd, a.qdm, a.x, \
                      a.xg, a.y, a.yg, b, a.lane_flags, a.part, a.treg, a.part_stride, a.lmap, a.qp)
         // every block a lattice brick: the two-waves-per-SIMD lattice kernel; else per element
         // (p = 2; at p = 1 the per-element kernel fits two waves already)
#define ECM2_TLB(RM)                                                                                          \
   hipLaunchKernelGGL((k_apply_tpe_tlb<3, 4, SPLIT, RM, PW>), grid, block, 0, s, a.ne, a.blk_begin, a.blk_end,      \
                      a.n_owned, a.gmap, a.qdd, a.qdm, a.x, a.xg, a.y, a.yg, b, a.lane_flags, a.part, a.treg,      \
                      a.part_stride, a.lmap, a.qp)
         constexpr bool LAT = D == 3 && Q == 4;
         if (LAT && a.treg && a.treg_all) { ECM2_TLB(1); }
         else if (LAT && a.treg && a.tlat_all) { ECM2_TLB(3); }
#undef ECM2_TLB
         else if (a.treg) { ECM2_TL((k_apply_tpe_sf<D, Q, SPLIT, 2, true, PW>)); }
         else { ECM2_TL((k_apply_tpe_sf<D, Q, SPLIT, 0, true, PW>)); }
#undef ECM2_TL
      }
      else { ECM2_VERIFY(false, ERR_INTERNAL, "TRILINEAR qdata needs the diffusion integrator"); }
      return;
   }
   if (a.kind == QLAYOUT_AFFINE && a.tsnap)
   {
      // the diffusion coefficient from its field snapshot: W alpha det J per point (tmass 1), or no
      // per-point stream (tmass 2)
      if constexpr (DIFF && D == 3 && Q == 4)
      {
         ECM2_VERIFY(a.tmass == (MASS ? a.tmass : 0) && (a.tmass != 0) == MASS && a.pw == (a.tmass == 1 ? 1 : 0) &&
                        a.treg && (a.treg_all || a.tlat_all) && a.tsnap_kind == (a.treg_all ? 1 : 2),
                     ERR_INTERNAL, "coefficient snapshot needs lattice blocks and matching mass values");
         Basis1D bw = b;  // (w B): the weight-scaled interpolation of T' (LAW = false)
         for (int d = 0; d < MAX_D1D; d++)
            for (int q = 0; q < MAX_Q1D; q++) { bw.B[q + MQ * d] = a.qw[q] * b.B[q + MQ * d]; }
         QPts qw = {};
         for (int q = 0; q < MAX_Q1D; q++) { qw.x[q] = a.qw[q]; }
#define ECM2_TS(RM, MM, LAW, CD)                                                                                    \
   hipLaunchKernelGGL((k_apply_tpe_ts<3, 4, SPLIT, RM, MM, LAW, CD>), grid, block, 0, s, a.ne, a.blk_begin, a.blk_end, \
                      a.n_owned, a.gmap, a.qdd, a.qdm, a.x, a.xg, a.tsnap, a.y, a.yg, b, bw, a.lane_flags, a.part,     \
                      a.treg, a.part_stride, a.lmap, qw, a.law_d, a.law_m, a.en)
#define ECM2_TS_MM(RM, LAW, CD)                                                                                     \
   if (!MASS) { ECM2_TS(RM, 0, LAW, CD); }                                                                          \
   else if (a.tmass == 1) { ECM2_TS(RM, 1, LAW, CD); }                                                              \
   else { ECM2_TS(RM, 2, LAW, CD); }
#define ECM2_TS_LAW(RM, CD)                                                                                         \
   if (a.tlaw) { ECM2_TS_MM(RM, true, CD) } else { ECM2_TS_MM(RM, false, CD) }
         // (axis-aligned meshes: the diagonal flux product, a.cdiag)
         if (a.treg_all)
         {
            if (a.cdiag) { ECM2_TS_LAW(1, true) } else { ECM2_TS_LAW(1, false) }
         }
         else
         {
            if (a.cdiag) { ECM2_TS_LAW(3, true) } else { ECM2_TS_LAW(3, false) }
         }
#undef ECM2_TS_LAW
#undef ECM2_TS_MM
#undef ECM2_TS
      }
      else { ECM2_VERIFY(false, ERR_INTERNAL, "coefficient snapshot: p = 2 forms with the diffusion integrator"); }
      return;
   }
   if (a.kind == QLAYOUT_AFFINE)
   {
      if constexpr (DIFF)
      {
         ECM2_VERIFY(a.pw == PW, ERR_INTERNAL, "AFFINE point values do not match the integrators");
         if (MASS && a.latency)
         {
            hipLaunchKernelGGL((k_apply_tpe_pp<D, Q, SPLIT>), dim3(nb), dim3(256), 0, s, a.ne, a.blk_begin,
                               a.n_owned, a.gmap, a.qdd, a.qdm, a.x, a.xg, a.y, a.yg, b, a.lane_flags, a.part,
                               a.part_stride);
         }
         else
         {
#define ECM2_SF(RM)                                                                                           \
   hipLaunchKernelGGL((k_apply_tpe_sf<D, Q, SPLIT, RM, false, PW>), grid, block, 0, s, a.ne, a.blk_begin, a.blk_end, \
                      a.n_owned, a.gmap, a.qdd, a.qdm, a.x, a.xg, a.y, a.yg, b, a.lane_flags, a.part, a.treg,       \
                      a.part_stride, a.lmap, a.qp)
            if (a.treg && a.treg_all) { ECM2_SF(1); }
            else if (a.treg && a.tlat_all) { ECM2_SF(3); }
            else if (a.treg) { ECM2_SF(2); }
            else { ECM2_SF(0); }
#undef ECM2_SF
         }
      }
      else { ECM2_VERIFY(false, ERR_INTERNAL, "AFFINE qdata needs the diffusion integrator"); }
      return;
   }
   hipLaunchKernelGGL((k_apply_tpe_pf<D, Q, MASS, DIFF, SPLIT>), grid, block, 0, s, a.ne, a.blk_begin, a.blk_end,
                      a.n_owned, a.gmap, a.qdd, a.qdm, a.x, a.xg, a.y, a.yg, b, rowtab, a.lane_flags, a.part);
}

template <int D, int Q, bool MASS, bool DIFF>
void launch_tpe_mdq(const ApplyArgs &a, const Basis1D &b, const double *rowtab, hipStream_t s)
{
   if (a.blk_end <= a.blk_begin) { return; }
   ECM2_VERIFY(a.lane_flags, ERR_INTERNAL, "thread-per-element kernel needs the merge plan");
   if (a.xg || a.yg) { launch_tpe<D, Q, MASS, DIFF, true>(a, b, rowtab, s); }
   else { launch_tpe<D, Q, MASS, DIFF, false>(a, b, rowtab, s); }
}

template <int D, int Q>
void launch_tpe_dq(bool mass, bool diff, const ApplyArgs &a, const Basis1D &b, const double *rowtab, hipStream_t s)
{
   if (mass && diff) { launch_tpe_mdq<D, Q, true, true>(a, b, rowtab, s); }
   else if (mass) { launch_tpe_mdq<D, Q, true, false>(a, b, rowtab, s); }
   else if (diff) { launch_tpe_mdq<D, Q, false, true>(a, b, rowtab, s); }
}

template <int D, int Q, bool MASS, bool DIFF>
void launch_diag_tpe(const ApplyArgs &a, const Basis1D &b, const double *drow, hipStream_t s)
{
   const int nb = a.blk_end - a.blk_begin;
   if (nb <= 0) { return; }
   const dim3 grid((nb + 3) / 4), block(256);
#define ECM2_DIAG(SP, AF, XV)                                                                            \
   hipLaunchKernelGGL((k_diag_tpe<D, Q, MASS, DIFF, SP, AF, XV>), grid, block, 0, s, a.ne, a.blk_begin,        \
                      a.blk_end, a.n_owned, a.gmap, a.qdd, a.qdm, a.y, a.yg, b, drow, a.lane_flags, a.part,  \
                      XV ? a.treg : nullptr, a.part_stride, XV ? a.lmap : nullptr)
   const bool aff = a.kind == QLAYOUT_AFFINE;
   // a.xwave: the plan was built with cross-wave faces (AFFINE or TRILINEAR forms)
   const bool xw = aff || a.xwave;
   ECM2_VERIFY(!aff || (MASS && DIFF), ERR_INTERNAL, "AFFINE qdata needs both integrators");
   if (a.yg)
   {
      if (aff) { ECM2_DIAG(true, true, true); }
      else if (xw) { ECM2_DIAG(true, false, true); }
      else { ECM2_DIAG(true, false, false); }
   }
   else
   {
      if (aff) { ECM2_DIAG(false, true, true); }
      else if (xw) { ECM2_DIAG(false, false, true); }
      else { ECM2_DIAG(false, false, false); }
   }
#undef ECM2_DIAG
}

template <int D, int Q>
void launch_diag_tpe_dq(bool mass, bool diff, const ApplyArgs &a, const Basis1D &b, const double *drow,
                        hipStream_t s)
{
   if (mass && diff) { launch_diag_tpe<D, Q, true, true>(a, b, drow, s); }
   else if (mass) { launch_diag_tpe<D, Q, true, false>(a, b, drow, s); }
   else if (diff) { launch_diag_tpe<D, Q, false, true>(a, b, drow, s); }
}

} // namespace

namespace kern
{

void apply_tpe(int D, int Q, bool mass, bool diff, const ApplyArgs &a, const Basis1D &b,
               const double *rowtab, hipStream_t s)
{
   if (a.ne == 0) { return; }
   if (D == 2 && Q == 3) { launch_tpe_dq<2, 3>(mass, diff, a, b, rowtab, s); }
   else if (D == 3 && Q == 4) { launch_tpe_dq<3, 4>(mass, diff, a, b, rowtab, s); }
   else { ECM2_VERIFY(false, ERR_UNSUPPORTED, "no thread-per-element kernel for D1D=" << D << " Q1D=" << Q); }
   ECM2_HIP(hipGetLastError());
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

} // namespace kern
} // namespace ecm2
