// kernels.hpp -- host launchers for the gfx950 HIP kernels (k_setup.hip: qdata and
// coefficient setup; k_tpe.hip: thread-per-element p <= 2 apply and diagonal; k_line.hip:
// line / brick p >= 3 apply and the sum-factorised diagonal; k_misc.hip: workgroup-per-element
// apply, restriction, vector and solver kernels).
//
// Quadrature-data layouts (the qdata a PA form owns):
//  * BLOCKED (fused thread-per-element kernel): elements in blocks of 64 (one
//    wave; lane = element).  The blocked element->dof map packs bit 30 = "shared dof"
//    (held by more than one entry after in-wave assembly: written to its partial slot,
//    or atomically added) and bit 31 = orientation sign.
//    diffusion qdata: [blk][q][pair 0..2][lane][2] holding the
//    symmetric entries (11,12),(13,22),(23,33); mass: [blk][q/2][lane][2] (two
//    consecutive quadrature points per 16-byte slot).  Every wave-instruction
//    is one 1 KiB contiguous dwordx4 load.
//  * AFFINE (fused thread-per-element kernel on meshes whose elements are all
//    parallelepipeds, with both integrators present): the same 64-element blocks, but
//    the geometry is stored once per element.  For an affine element J is constant, so
//    the reference's D(q) = W_q beta_q adj(J) adj(J)^T / det J factors into a per-point
//    scalar W_q beta_q times a per-element symmetric matrix C = adj(J) adj(J)^T / det J.
//    qd_diff holds C: [blk][pair 0..2][lane][2] (pairs (11,12),(13,22),(23,33));
//    qd_mass holds the per-point pair [blk][q][lane][2] = (W_q beta_q, W_q alpha_q det J).
//    16 B per quadrature point + 48 B per element instead of 56 B per point (3.3x fewer
//    qdata bytes at p = 2); the values are the reference's up to rounding.
//  * AFFINE_E (line / brick kernels, p >= 3, same conditions): caller element order,
//    qd_diff = C as [e][6] (11,12,13,22,23,33), qd_mass = pairs [e][q][2] (3.5x fewer
//    qdata bytes at p = 4).
//  * NATIVE (the reference's own layout): diffusion D(q,s,e) = [e][6][NQ],
//    mass v(q,e) = [e][NQ] (bilininteg_diffusion_kernels.cpp:356-361,
//    bilininteg_mass_pa.cpp:66-77).
#pragma once

#include "common.hpp"
#include "fe.hpp"

namespace ecm2
{

enum QLayoutKind : int { QLAYOUT_NATIVE = 0, QLAYOUT_BLOCKED = 1, QLAYOUT_AFFINE = 2, QLAYOUT_AFFINE_E = 3,
                         QLAYOUT_TRILINEAR = 4, QLAYOUT_NATIVE9 = 5, QLAYOUT_TRILINEAR_E = 6 };
// TRILINEAR_E: the TRILINEAR compression for the p >= 3 line / brick kernels, caller element
// order: qd_diff = [e][21] map coefficients c1..c7 of x, y, z (index 3 (k - 1) + i), qd_mass =
// [e][q][pw] point values.  AFFINE_E / TRILINEAR_E with pw = 1: a diffusion-only form.
// NATIVE9: the reference's layout for a general (nonsymmetric) matrix diffusion coefficient,
// D(q, k, e) = [e][9][NQ] with k = 3 i + j for D_ij (bilininteg_diffusion_kernels.cpp:320-345,
// "symmetric ? 6 : 9"); the workgroup-per-element kernels read it.
// TRILINEAR (fused thread-per-element kernel, p <= 2, both integrators, geometry from element
// corners, elements NOT all parallelepipeds): the geometry is stored once per element as the
// coefficients of its trilinear map x_i(xi, eta, zeta) = c0 + c1 xi + c2 eta + c3 zeta +
// c4 xi eta + c5 xi zeta + c6 eta zeta + c7 xi eta zeta (the expansion of GeometricFactors'
// sum over the corners, mesh.cpp:15220-15273), and the kernel evaluates J, adj(J), det J at
// each quadrature point (PADiffusionSetup3D's algebra, bilininteg_diffusion_kernels.cpp:
// 349-362): qd_diff = [blk][11 pairs][lane][2] holding c1..c7 of x, y, z (index 3 (k - 1) + i,
// padded to 22), qd_mass = [blk][q][lane][2] = (W_q beta_q / det J_q, W_q alpha_q det J_q) (the
// setup evaluates det J once, so the apply needs no division).  16 B per point + 176 B per
// element instead of 56 B per point: the bytes of the AFFINE layout on a general trilinear mesh,
// for ~33 extra FP64 operations per point (adj(J) and its two products).
constexpr int kTrilinPairs = 11;
// 1D Gauss-Legendre points on [0, 1] (kernel argument: scalar loads)
struct QPts
{
   double x[MAX_Q1D];
};

constexpr int kElemBlock = 64;  // elements per wave in the blocked layout

struct QLayout
{
   int kind = QLAYOUT_NATIVE;
   int ne = 0, nq = 0;
   // AFFINE / TRILINEAR point values: 2 = the pair (diffusion factor, mass factor), 1 = the
   // diffusion factor alone (a form without a MassIntegrator: [blk][q][lane], 8 B per point)
   int pw = 2;
   // AFFINE (p = 2, lattice blocks) with the diffusion coefficient a law of an H1 field on the form's
   // space (grid-function coefficient kinds): the kernel interpolates a snapshot of the field
   // (ApplyArgs::tsnap) instead of reading W beta per point.
   // 1: the snapshot in dof order (regular blocks); 2: in the lattice-map blocks' slot order
   int tsnap = 0;
   // with tsnap, the mass: 0 none; 1 W alpha det J per point (pw = 1: a quadrature coefficient, or a
   // grid function other than the diffusion's field); 2 one value per element, (c alpha) det J (pw = 0:
   // alpha constant, folded in, or a law of the diffusion's own field, evaluated in the kernel)
   int tmass = 0;
   // with tsnap: 0 the (affine) diffusion law applied to the snapshot's dofs and the weight-scaled
   // interpolation gives W beta directly; 1 the snapshot is the field itself, interpolated at the point,
   // where the laws are applied (TransformedCoefficient::Eval, coefficient.cpp:262: any law, and the
   // mass law of the same field)
   int tlaw = 0;
   const int *pos = nullptr;  // device: caller element -> internal position (BLOCKED)
   const int *perm = nullptr; // device: internal position -> caller element (BLOCKED)
   size_t diff_size() const
   {
      if (kind == QLAYOUT_NATIVE) { return (size_t)ne * 6 * nq; }
      if (kind == QLAYOUT_NATIVE9) { return (size_t)ne * 9 * nq; }
      if (kind == QLAYOUT_AFFINE) { return (size_t)nblk() * 6 * kElemBlock; }
      if (kind == QLAYOUT_TRILINEAR) { return (size_t)nblk() * 2 * kTrilinPairs * kElemBlock; }
      if (kind == QLAYOUT_AFFINE_E) { return (size_t)ne * 6; }
      if (kind == QLAYOUT_TRILINEAR_E) { return (size_t)ne * 21; }
      return (size_t)nblk() * nq * 6 * kElemBlock;
   }
   size_t mass_size() const
   {
      if (kind == QLAYOUT_NATIVE || kind == QLAYOUT_NATIVE9) { return (size_t)ne * nq; }
      if (kind == QLAYOUT_AFFINE && tsnap && tmass == 2) { return (size_t)nblk() * kElemBlock; }  // [blk][lane]
      if (kind == QLAYOUT_AFFINE || kind == QLAYOUT_TRILINEAR) { return (size_t)nblk() * nq * pw * kElemBlock; }
      if (kind == QLAYOUT_AFFINE_E || kind == QLAYOUT_TRILINEAR_E) { return (size_t)ne * nq * pw; }
      return (size_t)nblk() * ((nq + 1) / 2) * 2 * kElemBlock;
   }
   int nblk() const { return (ne + kElemBlock - 1) / kElemBlock; }
   bool blocked() const { return kind == QLAYOUT_BLOCKED || kind == QLAYOUT_AFFINE || kind == QLAYOUT_TRILINEAR; }
   bool affine() const { return kind == QLAYOUT_AFFINE || kind == QLAYOUT_AFFINE_E; }
   bool trilinear() const { return kind == QLAYOUT_TRILINEAR || kind == QLAYOUT_TRILINEAR_E; }
   // the point values live in qd_mass (present with either integrator)
   bool compressed() const { return affine() || trilinear(); }
};

// Coefficient descriptor for qdata setup: constant, per-quadrature-point array
// ([e][q], CoefficientVector COMPRESSED storage, coefficient.cpp:2006-2180), or
// an affine function of an H1 grid function interpolated at the quadrature
// points: c = scale * (1 + slope * (T(x_q) - t_ref))  (GridFunctionCoefficient,
// coefficient.cpp:250-253, composed with the Pennes k(T) law).
// COEFF_GRIDFUNC_PERFUSION: the Pennes heat-capacity + perfusion term of the implicit
// stage's mass coefficient, alpha(T) = rho_c + gdt_cb * w_b(T) with the temperature-dependent
// perfusion w_b(T) = w0 * max(0, 1 + a (T - t0)) below the coagulation temperature t_stop and
// 0 at or above it (perfusion shut-down in ablated tissue).  p = (rho_c, gdt_cb, w0, a, t0, t_stop).
// Vector / matrix diffusion coefficients (DiffusionIntegrator(VectorCoefficient / MatrixCoefficient),
// PADiffusionSetup3D coeffDim 3 / 6 / 9, bilininteg_diffusion_kernels.cpp:297-348): QUAD_* device
// [ne][nq][dim], CONST_* the dim values in cv; dim 3 = diag(v), 6 = symmetric (11,12,13,22,23,33),
// 9 = general, row-major M(i,j) at 3 i + j (CoefficientVector::ProjectTranspose, coefficient.cpp:2093-2123).
// COEFF_GRIDFUNC: GridFunctionCoefficient (coefficient.cpp:250-253, qfunction.cpp:73-98), the H1 field's
// own value at the point (no law): e.g. ex16p's conductivity kappa + alpha u, formed at the dofs
// (examples/ex16p.cpp:450-466).
enum CoeffKind : int { COEFF_CONSTANT = 0, COEFF_QUAD = 1, COEFF_GRIDFUNC_AFFINE = 2, COEFF_GRIDFUNC_PERFUSION = 3,
                       COEFF_QUAD_VECTOR = 4, COEFF_QUAD_SYMMATRIX = 5, COEFF_QUAD_MATRIX = 6,
                       COEFF_CONST_VECTOR = 7, COEFF_CONST_SYMMATRIX = 8, COEFF_CONST_MATRIX = 9,
                       COEFF_GRIDFUNC = 10 };
struct CoeffDesc
{
   int kind = COEFF_CONSTANT;
   double value = 1.0;           // constant
   double cv[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};  // CONST_VECTOR / _SYMMATRIX / _MATRIX
   const double *quad = nullptr; // device [ne][nq] (QUAD) or [ne][nq][dim] (QUAD_VECTOR / _SYMMATRIX / _MATRIX)
   const double *lvec = nullptr; // device L-vector of T
   double scale = 1.0, slope = 0.0, t_ref = 0.0;  // GRIDFUNC_AFFINE
   double p[6] = {0, 0, 0, 0, 0, 0};              // GRIDFUNC_PERFUSION
   const double *emask = nullptr; // device [ne] element weights of an attribute-marked integrator (form-owned)
   bool gridfunc() const
   {
      return kind == COEFF_GRIDFUNC_AFFINE || kind == COEFF_GRIDFUNC_PERFUSION || kind == COEFF_GRIDFUNC;
   }
   // values per point: 1 scalar, 3 vector, 6 symmetric matrix, 9 general matrix
   int dim() const
   {
      switch (kind)
      {
         case COEFF_QUAD_VECTOR: case COEFF_CONST_VECTOR: return 3;
         case COEFF_QUAD_SYMMATRIX: case COEFF_CONST_SYMMATRIX: return 6;
         case COEFF_QUAD_MATRIX: case COEFF_CONST_MATRIX: return 9;
         default: return 1;
      }
   }
   bool quad_values() const { return kind == COEFF_QUAD || (kind >= COEFF_QUAD_VECTOR && kind <= COEFF_QUAD_MATRIX); }
};

struct CoeffParams  // kernel-argument copy of CoeffDesc::p
{
   double p[6];
};

// The temperature law of a grid-function coefficient at one point (device and host).
__host__ __device__ inline double coeff_law(int kind, double T, double scale, double slope, double t_ref,
                                            const double *p)
{
   if (kind == COEFF_GRIDFUNC) { return T; }
   if (kind == COEFF_GRIDFUNC_PERFUSION)
   {
      const double r = 1.0 + p[3] * (T - p[4]);
      const double wb = (T < p[5] && r > 0.0) ? p[2] * r : 0.0;
      return p[0] + p[1] * wb;
   }
   return scale * (1.0 + slope * (T - t_ref));
}

// A grid-function coefficient's law as a kernel argument (the coefficient snapshot applies it at the
// quadrature point), in one branch-free form covering every law kind:
//   law(T) = c0 + c1 T + c2 r(T),  r(T) = max(0, 1 + a (T - t0)) for T < t_stop, else 0;
// COEFF_GRIDFUNC: c1 = 1; _AFFINE: c0 = scale (1 - slope t_ref), c1 = scale slope; _PERFUSION: c0 = rho_c,
// c2 = gdt_cb w0 (coeff_law's algebra, regrouped); a constant folded into stored values: c0 = 1.
struct PointLaw
{
   double c0 = 1.0, c1 = 0.0, c2 = 0.0, a = 0.0, t0 = 0.0, t_stop = 0.0;
};
inline PointLaw point_law_of(const CoeffDesc &c)
{
   PointLaw l;
   if (c.kind == COEFF_GRIDFUNC) { l.c0 = 0.0; l.c1 = 1.0; }
   else if (c.kind == COEFF_GRIDFUNC_AFFINE) { l.c0 = c.scale * (1.0 - c.slope * c.t_ref); l.c1 = c.scale * c.slope; }
   else if (c.kind == COEFF_GRIDFUNC_PERFUSION)
   {
      l.c0 = c.p[0]; l.c2 = c.p[1] * c.p[2]; l.a = c.p[3]; l.t0 = c.p[4]; l.t_stop = c.p[5];
   }
   return l;
}
__host__ __device__ inline double point_law(const PointLaw &l, double T)
{
   const double r = 1.0 + l.a * (T - l.t0);
   const double w = (T < l.t_stop && r > 0.0) ? r : 0.0;
   return l.c0 + l.c1 * T + l.c2 * w;
}

// Arguments of one fused apply over element blocks [blk_begin, blk_end) (64 elements per
// block).  With a split L-vector (distributed form) dofs >= n_owned live in xg / yg.
struct ApplyArgs
{
   int kind = QLAYOUT_NATIVE;
   int pw = 2;                      // AFFINE / TRILINEAR point values (QLayout::pw)
   int ne = 0, blk_begin = 0, blk_end = 0, n_owned = 0;
   const int *pos = nullptr;        // element permutation (blocked layout), may be null
   const int *lane_flags = nullptr; // [blk][64]: in-wave face merge flags
   const int *treg = nullptr;       // device [blk][8]: 4x4x4 blocks (base, sx, sy, sz, face mask, -, -, flag: 1 regular, 2 lattice slots), or null
   int treg_all = 0;                // every block regular
   int tlat_all = 0;                // every block a lattice-map block (treg flag 2)
   int part_stride = 0;             // p <= 2 partial slots per block (27 * 64, or the lattice surface when treg_all)
   const int *lmap = nullptr;       // device [blk][tpe_lattice_points]: lattice-slot blocks' lattice maps, or null
   QPts qp = {};                    // TRILINEAR: the quadrature points
   // AFFINE with a coefficient snapshot (QLayout::tsnap): T' = A + B T at the form's L-vector dofs
   // (the diffusion coefficient's law applied to its field at Assemble) and the 1D Gauss weights
   const double *tsnap = nullptr;
   int tsnap_kind = 0;              // QLayout::tsnap
   int tmass = 0, tlaw = 0;         // QLayout::tmass, QLayout::tlaw
   int cdiag = 0;                   // snapshot forms: every element's C = adj(J) adj(J)^T / det J diagonal
   PointLaw law_d, law_m;           // tlaw = 1: the diffusion and mass laws at the point
   double qw[MAX_Q1D] = {};
   int xwave = 0;                   // the merge plan has cross-wave faces (AFFINE / TRILINEAR forms)
   const int *gmap = nullptr;
   const double *qdd = nullptr, *qdm = nullptr;
   const double *x = nullptr, *xg = nullptr;
   double *y = nullptr, *yg = nullptr;
   double *part = nullptr;          // partial slots of shared dofs (null: atomics)
   bool latency = false;            // TPE + AFFINE: one workgroup per block, a plane per wave (small ranges)
   const Basis1D *btab = nullptr;   // LINE / brick / diagonal: device copy of the (D1D, Q1D) tables
   const int *lelem = nullptr;      // LINE: device list of the elements outside bricks
   const int *lelem_off = nullptr;  // LINE: host [nblk + 1], listed elements of 64-element block b
   // LINE, brick part (p >= 3 on structured regions): bricks of 2 x 2 x brick_bz elements
   const int *belem = nullptr;      // device [nbrick][4 bz] element ids (qdata addressing)
   const int *bmap = nullptr;       // device [nbrick][NB] lattice map: dof | shared << 30
   const int *breg = nullptr;       // device [nbrick][8]: regular bricks (base, sx, sy, sz, face mask), or null
   const int *brick_off = nullptr;  // host [nblk + 1], bricks whose first element lies in block b
   int brick_bz = 0;                // 0: no bricks
   double *part_brick = nullptr;    // partial slots [nbrick][surface] of shared lattice points
   // k_apply_tpe_ts: the Mult's energy x^T A x as one partial per workgroup (en[workgroup]), or null
   double *en = nullptr;
};

// Partial-slot order of a brick's surface lattice points (2 x 2 x bz elements, lattice
// LX = LY = 2 D - 1, LZ = bz (D - 1) + 1), grouped by face so that the two holders of a
// face dof -- this brick's high face and the neighbour's low face -- list it at the same
// offset within their groups: [Z = 0 | Z = LZ-1 | Y = 0 | Y = LY-1 | X = 0 | X = LX-1],
// edges and corners in the first group that contains them.  -1 for interior points.
__host__ __device__ constexpr int lattice_surface_points(int LX, int LY, int LZ)
{
   return 2 * LX * LY + 2 * (LZ - 2) * LX + 2 * (LZ - 2) * (LY - 2);
}
__host__ __device__ constexpr int lattice_surface_index(int LX, int LY, int LZ, int X, int Y, int Z)
{
   if (Z == 0) { return Y * LX + X; }
   if (Z == LZ - 1) { return LX * LY + Y * LX + X; }
   const int b1 = 2 * LX * LY;
   if (Y == 0) { return b1 + (Z - 1) * LX + X; }
   if (Y == LY - 1) { return b1 + (LZ - 2) * LX + (Z - 1) * LX + X; }
   const int b2 = b1 + 2 * (LZ - 2) * LX;
   if (X == 0) { return b2 + (Z - 1) * (LY - 2) + (Y - 1); }
   if (X == LX - 1) { return b2 + (LZ - 2) * (LY - 2) + (Z - 1) * (LY - 2) + (Y - 1); }
   return -1;
}
// Brick partial slots: the same face groups, each group starting on a multiple of kBrickSlotAlign
// doubles (ECM2_BRICK_SLOT_ALIGN, an A/B build: 16 = every group on its own 128-B lines).
#ifndef ECM2_BRICK_SLOT_ALIGN
#define ECM2_BRICK_SLOT_ALIGN 1
#endif
constexpr int kBrickSlotAlign = ECM2_BRICK_SLOT_ALIGN;
__host__ __device__ constexpr int slot_align_up(int n) { return (n + kBrickSlotAlign - 1) / kBrickSlotAlign * kBrickSlotAlign; }
__host__ __device__ constexpr int brick_surface_points(int D, int bz)
{
   const int LX = 2 * D - 1, LY = LX, LZ = bz * (D - 1) + 1;
   return 2 * slot_align_up(LX * LY) + 2 * slot_align_up((LZ - 2) * LX) + 2 * slot_align_up((LZ - 2) * (LY - 2));
}
__host__ __device__ constexpr int brick_surface_index(int D, int bz, int X, int Y, int Z)
{
   const int LX = 2 * D - 1, LY = LX, LZ = bz * (D - 1) + 1;
   const int gz = slot_align_up(LX * LY), gy = slot_align_up((LZ - 2) * LX), gx = slot_align_up((LZ - 2) * (LY - 2));
   if (Z == 0) { return Y * LX + X; }
   if (Z == LZ - 1) { return gz + Y * LX + X; }
   if (Y == 0) { return 2 * gz + (Z - 1) * LX + X; }
   if (Y == LY - 1) { return 2 * gz + gy + (Z - 1) * LX + X; }
   if (X == 0) { return 2 * gz + 2 * gy + (Z - 1) * (LY - 2) + (Y - 1); }
   if (X == LX - 1) { return 2 * gz + 2 * gy + gx + (Z - 1) * (LY - 2) + (Y - 1); }
   return -1;
}
static_assert(kBrickSlotAlign != 1 || (brick_surface_points(5, 1) == lattice_surface_points(9, 9, 5) &&
                                       brick_surface_index(5, 1, 3, 4, 2) == lattice_surface_index(9, 9, 5, 3, 4, 2) &&
                                       brick_surface_index(5, 1, 8, 4, 2) == lattice_surface_index(9, 9, 5, 8, 4, 2)),
              "unaligned brick slots are the lattice's face-grouped order");
// the same for a p <= 2 block (4 x 4 x 4 elements, lattice 4 (D-1) + 1 per side)
__host__ __device__ inline int tpe_surface_points(int D)
{
   return lattice_surface_points(4 * D - 3, 4 * D - 3, 4 * D - 3);
}
__host__ __device__ inline int tpe_surface_index(int D, int X, int Y, int Z)
{
   return lattice_surface_index(4 * D - 3, 4 * D - 3, 4 * D - 3, X, Y, Z);
}

// Block lattice map (lattice-slot blocks): one entry per point of the block's (4(D-1)+1)^3
// lattice, in "parity-class" order: the points are grouped by (X, Y, Z) mod (D-1) -- the
// classes a lane's entry a = (dx, dy, dz) falls in -- and lexicographic within a class, so the 64
// lanes' loads of one entry a touch one contiguous 4 x 4 x 4 sub-block (coalesced) and every
// point is stored once (729 ints at p = 2 against 27 x 64 per-entry map ints).
__host__ __device__ constexpr int tpe_lattice_points(int D)
{
   return (4 * (D - 1) + 1) * (4 * (D - 1) + 1) * (4 * (D - 1) + 1);
}
// points of residue class c (mod D - 1) along one axis of the lattice
__host__ __device__ constexpr int tpe_lattice_class_n(int c) { return c == 0 ? 5 : 4; }
// first slot of residue class (cx, cy, cz): classes in (cz, cy, cx) lexicographic order
__host__ __device__ constexpr int tpe_lattice_class_off(int D, int cx, int cy, int cz)
{
   const int P = D - 1;
   int off = 0;
   for (int k = 0; k < cz; k++) { off += tpe_lattice_class_n(k) * (4 * P + 1) * (4 * P + 1); }  // whole earlier z-classes
   const int nz = tpe_lattice_class_n(cz);
   for (int j = 0; j < cy; j++) { off += nz * tpe_lattice_class_n(j) * (4 * P + 1); }
   const int ny = tpe_lattice_class_n(cy);
   for (int i = 0; i < cx; i++) { off += nz * ny * tpe_lattice_class_n(i); }
   return off;
}
__host__ __device__ constexpr int tpe_lattice_slot(int D, int X, int Y, int Z)
{
   const int P = D - 1;
   const int cx = X % P, cy = Y % P, cz = Z % P;
   const int ny = tpe_lattice_class_n(cy), nx = tpe_lattice_class_n(cx);
   return tpe_lattice_class_off(D, cx, cy, cz) + ((Z / P) * ny + (Y / P)) * nx + (X / P);
}

// LDS image of a p = 2 block lattice for 16-byte reads (k_apply_tpe_ts: an (x, T') pair per point).
// Lane (ex, ey, ez) of the plane loop reads class (cx, cy, cz) at ez sz + ey sy + ex plus a
// wave-uniform offset; ds_read_b128 serves a wave in four 16-lane groups ({0-3, 12-15, 20-27},
// {4-11, 16-19, 28-31} and the same +32), each conflict-free iff its 16 lanes hit 16 distinct 16-byte
// slots of a 256-byte bank row.  The compact class order (row stride nx, plane stride nx ny) maps
// them 2.5-way on average (10.2 LDS cycles per read against 4: the 13.2M conflict cycles per launch
// of profiles/r5/sq/sq_r5_c4_xcd.json are 108 reads x 6.2 x 19,683 waves).  With the row stride
// sy = 4 (nx = 4) or 8 (nx = 5) and the plane stride sz = 0 mod 16 (sy 4) or 4 mod 8 (sy 8) the
// four (ey, ez) rows of every group fall on the four distinct quarter-rows: 1,100 slots instead of
// 729, conflict-free (tsl_conflict_free below, checked at compile time).
__host__ __device__ constexpr int tsl_sy(int nx) { return nx == 5 ? 8 : 4; }
__host__ __device__ constexpr int tsl_sz(int nx, int ny) { return nx == 4 ? (ny == 4 ? 16 : 32) : (ny == 4 ? 36 : 44); }
__host__ __device__ constexpr int tsl_class_size(int cx, int cy, int cz)
{
   const int nx = tpe_lattice_class_n(cx), ny = tpe_lattice_class_n(cy), nz = tpe_lattice_class_n(cz);
   return tsl_sz(nx, ny) * (nz - 1) + tsl_sy(nx) * (ny - 1) + nx;
}
__host__ __device__ constexpr int tsl_class_off(int cx, int cy, int cz)
{
   int off = 0;
   for (int c = 0; c < ((cz * 2 + cy) * 2 + cx); c++) { off += tsl_class_size(c & 1, (c >> 1) & 1, c >> 2); }
   return off;
}
__host__ __device__ constexpr int tsl_points() { return tsl_class_off(0, 0, 2); }  // (all eight classes)
// slot of lattice point (X, Y, Z) (p = 2: classes mod 2)
__host__ __device__ constexpr int tsl_slot(int X, int Y, int Z)
{
   const int cx = X & 1, cy = Y & 1, nx = tpe_lattice_class_n(cx), ny = tpe_lattice_class_n(cy);
   return tsl_class_off(cx, cy, Z & 1) + (Z >> 1) * tsl_sz(nx, ny) + (Y >> 1) * tsl_sy(nx) + (X >> 1);
}
__host__ __device__ constexpr bool tsl_conflict_free()
{
   for (int r = 0; r < 27; r++)  // the plane loop's reads (dx, dy, dz)
   {
      const int dx = r % 3, dy = (r / 3) % 3, dz = r / 9;
      for (int g = 0; g < 4; g++)
      {
         bool used[16] = {};
         for (int lane = 0; lane < 64; lane++)
         {
            const int l = lane & 31;
            const int grp = (lane >> 5) * 2 + ((l < 4 || (l >= 12 && l < 16) || (l >= 20 && l < 28)) ? 0 : 1);
            if (grp != g) { continue; }
            const int s = tsl_slot(2 * (lane & 3) + dx, 2 * ((lane >> 2) & 3) + dy, 2 * (lane >> 4) + dz) & 15;
            if (used[s]) { return false; }
            used[s] = true;
         }
      }
   }
   return true;
}
static_assert(tsl_conflict_free(), "k_apply_tpe_ts lattice image: conflict-free 16-byte reads");
static_assert(tsl_points() == 1100, "padded lattice image size");

namespace kern
{
// ---- setup (S1/S2/S3 equivalents) ----
// Evaluate a grid-function coefficient at quadrature points into out[e][q]
// (GridFunctionCoefficient projection, qfunction.cpp:73-98, then the temperature law).
// btab: device copy of b (the sum-factorised kernel's tables).
void coeff_gridfunc(int ne, int D, int Q, const int *gmap_native, const Basis1D &b, const Basis1D *btab,
                    const CoeffDesc &c, double *out, hipStream_t s);
// qdata from lexicographic element corner coordinates enodes[e][3][8].
void setup_from_nodes(const QLayout &L, int Q, const double *enodes, const double *W,
                      const Basis1D &b1, const CoeffDesc *cm, const CoeffDesc *cd,
                      const double *cm_q, const double *cd_q,
                      double *qd_diff, double *qd_mass, hipStream_t s);
// AFFINE / AFFINE_E layout (see above) from the corners of parallelepiped elements; needs the
// diffusion coefficient (cd); cm null: a diffusion-only form (L.pw = 1, AFFINE only).
// J (optional, device, MFEM layout NQ x 3 x 3 x NE) replaces the corners.
// AFFINE (blocked) / AFFINE_E C factors: are all off-diagonal entries exactly zero (axis-aligned elements)?  dflag: one
// device int of scratch.  Synchronises the stream.
bool affine_c_diagonal(const QLayout &L, const double *qd_fac, int *dflag, hipStream_t s);
void setup_affine(const QLayout &L, int Q, const double *enodes, const double *J, const double *W,
                  const CoeffDesc *cm, const CoeffDesc *cd, const double *cm_q, const double *cd_q,
                  double *qd_fac, double *qd_pair, hipStream_t s);
// TRILINEAR layout (see above) from lexicographic element corners; cd, and cm unless L.pw = 1.
// (enodes: lexicographic corners, or cfit: the fitted map coefficients [ne][21] of
// jacobians_trilinear_fit)
void setup_trilinear(const QLayout &L, int Q, const double *enodes, const double *cfit, const double *W,
                     const QPts &qp, const CoeffDesc *cm, const CoeffDesc *cd, const double *cm_q, const double *cd_q,
                     double *qd_geo, double *qd_pair, hipStream_t s);
// Trilinear-map coefficients of every element from MFEM-layout Jacobians (cfit [ne][21]); false
// when some element's Jacobians are not those of a trilinear map (1e-13; synchronises s).
// The BLOCKED per-point qdata of an AFFINE coefficient-snapshot form (p = 2): D = W beta_q C_e from the
// stored element matrices (qd_fac) and beta at the points (device [ne][nq], caller order); the mass from
// the stored values qd_m (per point, or per element times W_q alpha_q; alpha_q null: 1).
void tsnap_expand(const QLayout &L, int Q, const double *W, const double *qd_fac, const double *qd_m,
                  const double *beta_q, const double *alpha_q, double *qd_diff, double *qd_mass, hipStream_t s);
// Multiply integrator `integ`'s (0 mass, 1 diffusion) stored qdata on caller element e by w[e]
// (device [ne]), in any layout L (pos: L.pos for the blocked layouts).
void scale_elements(const QLayout &L, int integ, const double *w, double *qd_diff, double *qd_mass, hipStream_t s);
// out[i] = A + B T[i] (i < n): the coefficient snapshot of an affine law of an H1 field.
void affine_snapshot(int n, const double *T, double A, double B, double *out, hipStream_t s);
// The snapshot in the lattice-map blocks' slot order ([blk][nlp], lmap: the blocks' lattice maps),
// and its values back in dof order.
void affine_snapshot_lattice(int nblk, int nlp, const int *lmap, const double *T, double A, double B, double *out,
                             hipStream_t s);
void lattice_to_dofs(int nblk, int nlp, const int *lmap, const double *v, double *out, hipStream_t s);
bool jacobians_trilinear_fit(int ne, int Q, const QPts &qp, const double *J, double *cfit, hipStream_t s);
// The BLOCKED per-point qdata of an AFFINE (p <= 2) form (L: its layout; outputs sized as BLOCKED).
void affine_expand(const QLayout &L, int Q, const double *qd_fac, const double *qd_pair, double *qd_diff,
                   double *qd_mass, hipStream_t s, const double *qm1 = nullptr);
// The BLOCKED per-point qdata of a TRILINEAR form (L: its layout; outputs sized as BLOCKED).
void trilinear_expand(const QLayout &L, int Q, const double *qd_geo, const double *qd_pair, const QPts &qp,
                      double *qd_diff, double *qd_mass, hipStream_t s);
// Every element's Jacobian the same at all its points (1e-13 relative; synchronises s).
bool jacobians_affine(int ne, int nq, const double *J, hipStream_t s);
// qdata from MFEM-layout Jacobians J(q,i,j,e) (GeometricFactors::JACOBIANS).
void setup_from_jacobians(const QLayout &L, const double *J, const double *W,
                          const CoeffDesc *cm, const CoeffDesc *cd,
                          const double *cm_q, const double *cd_q,
                          double *qd_diff, double *qd_mass, hipStream_t s);

// ---- apply ----
// Fused y = R^T (M + K) R x, thread-per-element (blocked layout); y must be zeroed.
void apply_tpe(int D, int Q, bool mass, bool diff, const ApplyArgs &a, const Basis1D &b,
               const double *rowtab, hipStream_t s);
// Row table for apply_tpe: [qz][qy][3][dz][dy] products (see k_tpe.hip).
std::vector<double> make_row_table(const DofToQuad &m);
// Line kernel: one wave per listed element (a.lelem), native or AFFINE_E qdata, L-vectors
// through an encoded map [e][nd] (dof | shared << 30 | sign << 31); shared dofs go to
// part[e*nd + a] when a.part is set, else atomics; then the bricks (a.brick_bz).
// has_line: (D, Q) instantiated.
bool has_line(int D, int Q);
void apply_line(int D, int Q, bool mass, bool diff, const ApplyArgs &a, hipStream_t s);
// Brick kernel of the line family: (D, Q, bz) instantiated?  Lattice points per brick.
bool has_brick(int D, int Q, int bz);
int brick_points(int D, int bz);
// Workgroup-per-element kernel, any layout; in/out either L-vectors (through the
// gather map; output by atomics into a zeroed y) or E-vectors (accumulated).
void apply_wpe(int D, int Q, bool mass, bool diff, const ApplyArgs &a, bool in_evec,
               bool out_evec, const Basis1D &b, hipStream_t s);

// ---- ElementRestriction ----
void restriction_mult(long n, int nd, const int *gmap_native, const double *x, double *xe,
                      hipStream_t s);
void restriction_mult_transpose(int ndofs, int nd, const int *offsets, const int *indices,
                                const double *xe, double *y, hipStream_t s);

// ---- diagonal (Jacobi) ----
// Thread-per-element diagonal on the blocked layout, assembled/stored like apply_tpe (a.y /
// a.yg / a.part / a.lane_flags; a.x unused); drow = make_diag_row_table.
void diagonal_tpe(int D, int Q, bool mass, bool diff, const ApplyArgs &a, const Basis1D &b, const double *drow,
                  hipStream_t s);
std::vector<double> make_diag_row_table(const DofToQuad &m);
// Sum-factorised workgroup-per-element diagonal, any layout; L-vector (atomics) or E-vector.
void diagonal(const int *pos, int D, int Q, int layout, int ne, const int *gmap_native, const double *qd_diff,
              const double *qd_mass, double *diag, bool out_evec, const Basis1D &b, const Basis1D *btab,
              hipStream_t s);

// ---- vector kernels for the device PCG ----
void set_values(int n, const int *idx, double val, double *y, hipStream_t s);     // y[idx] = val
void copy_values(int n, const int *idx, const double *x, double *y, hipStream_t s); // y[idx] = x[idx]
// The device-driven PCG loop's state (device memory; the check kernels also write it to a mapped
// pinned host mirror): done = PCG_RUNNING or the stop code below; iters, final = the iteration
// (CGSolver's final_iter) and (B r, r) at which it stopped; checked (mirror) = the last iteration whose
// betanom test ran.  The vector kernels of an iteration given `ctl` return at once when done is set,
// so the host can enqueue an iteration before it has read the previous one's test.
struct PcgCtl
{
   int done, iters, checked, pad;
   double final;
};
// stop codes (CGSolver::Mult, solvers.cpp:950-1004): converged; max_iter reached; (B r, r) < 0 (the
// preconditioner is not positive definite: not converged); (A d, d) == 0 (not converged); a
// non-finite (B r, r) or (A d, d) (MFEM_VERIFY(IsFinite) aborts: ECM2_ERR_NUMERIC)
enum PcgDone
{
   PCG_RUNNING = 0,
   PCG_CONVERGED = 1,
   PCG_MAX_ITER = 2,
   PCG_NEG_BR = 3,
   PCG_DEN_ZERO = 4,
   PCG_NONFINITE = 5
};
// A stopping test on the device.  kind 0: iteration `it`'s test of betanom = the dot (non-finite,
// < 0, <= r0, it + 1 > max_iter); kind 1: the test of den = the dot in iteration it - 1's tail (it =
// the incremented iteration number, CGSolver's final_iter on a den == 0 stop; final = *betanom).
// Writes ctl and the host mirror once, when done is first set.
struct PcgStop
{
   double r0;
   int it, max_iter;
   PcgCtl *ctl, *host;
   const double *betanom = nullptr;
   int kind = 0;
};
// Deterministic two-pass dot: result written to *out (device).  partials: max(step_parts(n), kDotPartials).
// hout (optional): device pointer of mapped pinned host memory that also receives the result.
// stop (serial solver): a stopping test on *out in the same launch.
constexpr int kDotPartials = 1024;
void dot(int n, const double *a, const double *b, double *partials, double *out, hipStream_t s,
         double *hout = nullptr, const PcgCtl *ctl = nullptr, const PcgStop *stop = nullptr);
// CGSolver's update in two passes (4 + 6 vector streams, z never stored):
//   pcg_step_r: alpha = nom/den (-> *alpha); r -= alpha z (z holds A d); *out = r.(dinv .* r)
//               (r.r without dinv), deterministic; stop (serial): betanom test in the same launch;
//   pcg_update_xd: x += (nom/den) d; d = dinv .* r + (betanom/nom) d;
//   pcg_finish_x (after the loop): x += *alpha d if the loop stopped at a betanom test.
// the partial sums of dot's first pass (one per workgroup of its flat grid; pcg_step_r writes kDotPartials):
// the partials buffer must hold them
int step_parts(int n);
void pcg_step_r(int n, const double *nom, const double *den, const double *z, double *r, const double *dinv,
                double *partials, double *out, double *alpha, hipStream_t s, const PcgCtl *ctl = nullptr,
                const PcgStop *stop = nullptr);
void pcg_update_xd(int n, const double *nom, const double *den, const double *betanom, double *x, double *d,
                   const double *r, const double *dinv, hipStream_t s, const PcgCtl *ctl = nullptr);
void pcg_finish_x(int n, const double *alpha, const double *d, double *x, hipStream_t s, const PcgCtl *ctl);
// a stopping test alone (after a distributed dot's all-reduce)
void pcg_check(const double *v, const PcgStop &stop, hipStream_t s);
// saved[i] = v[idx[i]], v[idx[i]] = 0  /  v[idx[i]] = y[idx[i]] = saved[i]
void ess_save_zero(int n, const int *idx, double *v, double *saved, hipStream_t s);
void ess_restore(int n, const int *idx, const double *saved, double *v, double *y, hipStream_t s,
                 double *sq_parts = nullptr);
// ess_restore's blocks: sq_parts[block] = the block's sum of saved^2 (fixed order), ess_parts(n) of them
int ess_parts(int n);
// the second pass of a deterministic dot over nparts given partials (+ optional stopping test)
void dot_final(int nparts, const double *partials, double *out, hipStream_t s, const PcgCtl *ctl = nullptr,
               const PcgStop *stop = nullptr, double *hout = nullptr);
//   z = dinv .* r  (dinv may be null -> z = r)
void pcg_precond(int n, const double *dinv, const double *r, double *z, hipStream_t s);
void reciprocal(int n, const double *a, double *out, hipStream_t s);
void scale(int n, double a, double *y, hipStream_t s);                                   // y *= a
void add_scaled(int n, const double *x, double c, const double *k, double *out, hipStream_t s); // out = x + c k
// b = a with 16-byte nontemporal accesses (HBM STREAM-copy measurement)
void stream_copy(long n, const double *a, double *b, hipStream_t s);
// read-only stream: out[t] = sum of thread t's 16-byte loads (nout >= the launch's threads)
void stream_read(long n, const double *a, double *out, long nout, hipStream_t s);
// Halo pack/unpack for the distributed operator (K7): buf[i] = x[idx[i]] ; y[idx[i]] += buf[i]
void gather_idx(int n, const int *idx, const double *x, double *buf, hipStream_t s);
void scatter_add_idx(int n, const int *idx, const double *buf, double *y, hipStream_t s);
// Deterministic second scatter pass, run-compressed (PAForm::build_shared_plan), over plan
// blocks [b0, b1): block k sums the entries of runs [blocks[2k], blocks[2k+1]) (<= 256 entries).
// Run r = runs[r][12] = {n1 | n2 << 8 | cnt << 16, dof0, d1, d2, t1, t2, entry0, slot_off,
// s0, s1, s2, s3}: its entry at lattice position (a, b) (offset a + n1 b from entry0) stores
// y[dof0 + a d1 + b d2] = sum over holders h < cnt (ascending slots) of part[s_h + a t1 + b t2],
// s_h = runs[r][8 + h] for h < 4, else rslots[slot_off + h].  runs has a sentinel row.
void sum_partials(int b0, int b1, const int *blocks, const int *runs, const int *rslots, const int *pdof, const double *part,
                  int n_owned, double *y, double *yg, hipStream_t s);
} // namespace kern

} // namespace ecm2
