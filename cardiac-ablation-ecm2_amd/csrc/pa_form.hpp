// pa_form.hpp -- MI355X PA form: the drop-in for the reference's
// BilinearForm(PARTIAL) + {MassIntegrator(alpha), DiffusionIntegrator(beta)}
// and its PABilinearFormExtension.
//
// Reference interface mirrored:
//   PABilinearFormExtension::Assemble / Mult / AssembleDiagonal
//                                          fem/bilinearform_ext.hpp:67-144, .cpp:332-564
//   BilinearFormIntegrator::AssemblePA / AddMultPA / AssembleDiagonalPA
//                                          fem/bilininteg.hpp:49-97
//   ElementRestriction::Mult / MultTranspose fem/restriction.cpp:109-186
// Ownership follows the reference: the form owns qdata and its work vectors;
// x / y are caller-owned device arrays; all work is enqueued on the caller's
// stream (the reference uses the null stream, forall.hpp:782).
#pragma once

#include "common.hpp"
#include "fe.hpp"
#include "kernels.hpp"

#include <memory>
#include <utility>
#include <vector>

namespace ecm2
{

enum KernelMode : int
{
   KERNEL_AUTO = 0,     // TPE for p = 1, 2; LINE for p = 3..6; else WPE
   KERNEL_TPE = 1,      // fused, thread per element (p = 1, 2)
   KERNEL_WPE = 2,      // fused, workgroup per element, all intermediates in LDS (any p)
   KERNEL_UNFUSED = 3,  // reference-shaped: restriction, per-integrator AddMultPA, CSR transpose
   KERNEL_LINE = 4      // fused, one wave per element, register lines (Q1D <= 8)
};

// How the fused TPE kernel combines contributions to dofs held by more than one element
// entry (after in-wave face assembly):
enum ScatterMode : int
{
   SCATTER_PARTIALS = 0,  // dense partial slots + a fixed-order summation pass (deterministic)
   SCATTER_ATOMIC = 1     // FP64 atomic adds into a zeroed y
};

enum IntegratorKind : int { INTEG_MASS = 0, INTEG_DIFFUSION = 1 };

class PAForm
{
public:
   // n_owned < ndofs: the local L-vector is split [owned | ghost] (distributed form);
   // x/y hold dofs < n_owned, xg/yg the ghosts (apply_blocks).
   PAForm(int ne, int order, int ndofs, const int *gather_map_host, int q1d = 0, int n_owned = -1);
   ~PAForm();

   int ne() const { return ne_; }
   int order() const { return order_; }
   int ndofs() const { return ndofs_; }
   int d1d() const { return D_; }
   int q1d() const { return Q_; }
   int layout() const { return layout_.kind; }
   int kernel_mode() const { return resolved_mode_; }

   // Geometry: lexicographic corner coordinates (host, [ne][3][8]) or
   // MFEM-layout Jacobians (device, NQ x 3 x 3 x NE; the pointer must stay
   // valid until assemble()).
   void set_element_nodes(const double *enodes_host);
   void set_jacobians(const double *J_device);
   // AFFINE qdata (kernels.hpp) for the fused p <= 2 kernel when every element is a
   // parallelepiped (checked on the corners) and both integrators are present: on by default.
   void set_geometry_compression(bool on);
   bool affine_geometry() const { return affine_; }
   // Coefficient snapshot (AFFINE, p = 2, lattice blocks, the diffusion coefficient an affine law
   // of an H1 field, unmarked): the law applied to the field's dofs at Assemble and interpolated by
   // the kernel, instead of a stored W beta per point.  On by default; coefficient_snapshot() says
   // whether the last Assemble took it.
   void set_coefficient_snapshot(bool on);
   bool coefficient_snapshot() const { return layout_.tsnap != 0; }
   // with the snapshot: the mass values (QLayout::tmass) and where the laws are applied (QLayout::tlaw)
   int snapshot_mass() const { return layout_.tmass; }
   int snapshot_law_at_point() const { return layout_.tlaw; }
   bool flux_diagonal() const { return cdiag_ && (layout_.tsnap || layout_.kind == QLAYOUT_AFFINE_E); }
   // bytes of quadrature data the form stores (diffusion + mass + the coefficient snapshot)
   size_t qdata_bytes() const { return qd_diff_.bytes() + qd_mass_.bytes() + tsnap_.bytes(); }

   // Optional element permutation (internal position i <- caller element perm[i]) used by
   // the blocked layout; ORDER_BRICK puts one 4x4x4 brick in each 64-lane wave so the
   // fused kernel can assemble shared faces in-wave.  Without one, assemble() derives a
   // brick order from the element->dof map (face_brick_order, any conforming mesh).  All
   // APIs keep caller element order.
   void set_element_order(const int *perm_host);
   // Block indices at which apply_blocks ranges may start or end besides 0 and nblocks()
   // (the distributed form's interior | boundary split).  The line kernel's bricks never
   // straddle one.
   void set_block_splits(const std::vector<int> &splits);
   // Bricks of the line kernel family (p >= 3, both integrators, partial scatter): -1 =
   // default (2 x 2 x 1), 0 = none, 1 = 2 x 2 x 1, 2 = 2 x 2 x 2 elements per workgroup.
   void set_line_bricks(int bz);
   // Blocks >= b are applied with the one-block-per-workgroup latency kernel (apply_blocks
   // latency = true): no cross-wave face assembly there.  -1: none.
   void set_latency_from(int b);
   int n_bricks() const { return n_bricks_; }
   // units (p <= 2 blocks, p >= 3 bricks) whose dofs the fused kernel computes from 5 ints
   // instead of reading the map
   int lattice_units() const
   {
      if (resolved_mode_ == KERNEL_TPE)
      {
         return (layout_.kind == QLAYOUT_AFFINE || layout_.kind == QLAYOUT_TRILINEAR) ? n_treg_ : 0;
      }
      return (resolved_mode_ == KERNEL_LINE && breg_.size()) ? n_bricks_ : 0;
   }
   int n_units() const { return resolved_mode_ == KERNEL_TPE ? layout_.nblk() : n_bricks_; }
   // p <= 2 blocks with face-grouped partial slots but map-addressed dofs (a numbering that is not a lattice)
   int lattice_slot_units() const { return resolved_mode_ == KERNEL_TPE ? n_tlat_ : 0; }
   int brick_bz() const { return brick_bz_; }
   // BilinearForm::AddDomainIntegrator(integ[, elem_marker]) (bilinearform.cpp:231-242): with a
   // marker (host marker[n_marker], 0 / 1 per attribute), the integrator acts on the elements
   // whose attribute a has a > 0 and marker[a - 1] != 0 only (AddMultWithMarkers,
   // bilinearform_ext.cpp:753-774,807-847); the attributes come from set_attributes.
   void add_integrator(int kind, const CoeffDesc &c, const int *marker = nullptr, int n_marker = 0);
   // element attributes (host [ne], caller element order), as Mesh::GetAttribute
   void set_attributes(const int *attr_host);
   void set_kernel(int mode);
   void set_scatter(int mode);
   int scatter() const { return scatter_; }
   bool use_partials() const
   {
      return (resolved_mode_ == KERNEL_TPE || resolved_mode_ == KERNEL_LINE) && scatter_ == SCATTER_PARTIALS;
   }
   void assemble(hipStream_t s);

   // y = A x (BilinearForm::Mult semantics: y overwritten).
   void mult(const double *x, double *y, hipStream_t s);
   // y += a A x (Operator::AddMult, linalg/operator.hpp:87-92): Mult into a form-owned work
   // vector, then one axpy.  Like every call on a form (the reference's Mult reuses its
   // localX / localY too, bilinearform_ext.hpp:75), AddMult is stream-serial per form: two calls
   // on the same form must be ordered (same stream or an event), not run concurrently.
   void add_mult(const double *x, double *y, double a, hipStream_t s);
   // The Mult with its energy x^T A x folded in (CGSolver's den = (A d, d), solvers.cpp:993, without
   // a dot pass over the vectors): energy_parts() partials (one per workgroup of the single apply
   // launch, summed in a fixed order by the caller) -- or 0 when this form's kernel does not fold it
   // (only the coefficient-snapshot kernel k_apply_tpe_ts does; the caller then runs the dot).
   int energy_parts() const;
   void mult_energy(const double *x, double *y, double *en, hipStream_t s);
   bool assembled() const { return assembled_; }
   // Incremented by every assemble(): whoever caches device pointers or launches of this form
   // (the distributed form's HIP graphs) rebuilds them when it changes.
   long generation() const { return gen_; }
   // Fused apply of element blocks [b0, b1) (64 elements per block); x / xg as in the
   // constructor's split.  Atomic scatter: accumulates into zero-initialised y / yg.
   // Partial scatter: stores the dofs held once, writes the shared ones' partial slots;
   // finish_shared over the shared-dof range [i0, i1) then stores those (the owned
   // shared dofs are [0, n_shared_owned()), the ghost ones [n_shared_owned(), n_shared())).
   // latency: small block range on a critical path (the p <= 2 AFFINE kernel then gives each
   // block a workgroup with one quadrature plane per wave).
   void apply_blocks(const double *x, const double *xg, double *y, double *yg, int b0, int b1,
                     hipStream_t s, bool latency = false, double *en = nullptr);
   void finish_shared(int i0, int i1, double *y, double *yg, hipStream_t s);
   int n_shared() const { return n_sh_; }
   int n_shared_owned() const { return n_sh_owned_; }
   long n_partial_slots() const { return n_slots_; }
   long n_summation_runs() const { return n_runs_; }
   long n_explicit_runs() const { return n_explicit_runs_; }
   int nblocks() const { return layout_.nblk(); }
   bool has_mass() const { return have_mass_; }
   bool has_diffusion() const { return have_diff_; }
   void assemble_diagonal(double *diag, hipStream_t s);  // cached per assembly (gen_)

   // Reference-shaped pieces (E-vector layout [e][nd], lexicographic).
   void restriction_mult(const double *x, double *xe, hipStream_t s);
   void restriction_mult_transpose(const double *xe, double *y, hipStream_t s);
   void integrator_add_mult(int kind, const double *xe, double *ye, hipStream_t s);
   // qdata in the reference's native layout, copied to the host.
   void get_qdata(int kind, double *out_host, hipStream_t s);

   // HIP-event timing of the dominant (apply) kernel.
   void timing_enable(bool on);
   bool timing_on() const { return timing_; }
   void timing_get(double *total_ms, long *launches);
   size_t algorithmic_bytes() const;

private:
   void ensure_csr();
   void ensure_work(hipStream_t s);
   void record_start(hipStream_t s);
   void record_stop(hipStream_t s);
   // second pass of the deterministic scatter from the shared holding entries
   // (hdof[i], hslot[i]) in ascending slot order and the per-dof holder counts
   void build_shared_plan(const std::vector<int> &hcount, const std::vector<int> &hdof,
                          const std::vector<int> &hslot, hipStream_t s);
   ApplyArgs apply_args(const double *x, const double *xg, double *y, double *yg, int b0,
                        int b1) const;
   // qdata of the integrators present (resized, padding cleared, coefficients projected, setup
   // kernel)
   void setup_qdata(hipStream_t s);
   // element weights [ne] of integrator kind k: 1 / 0 per its attribute marker, all 1 unmarked
   std::vector<double> marker_weights(int k) const;
   void diagonal_from_qdata(double *diag, hipStream_t s);
   void assemble_diagonal_uncached(double *diag, hipStream_t s);
   // TRILINEAR(_E) forms and diffusion-only AFFINE(_E) forms: their per-point qdata in the BLOCKED
   // (p <= 2) or NATIVE (p >= 3) layout, expand_kind() (temporaries of the caller) for the
   // diagonal, the E-vector apply and the qdata export
   bool expand_needed() const
   {
      return layout_.trilinear() || layout_.tsnap || (layout_.affine() && layout_.pw == 1);
   }
   // coefficient values at the quadrature points ([e][q], tmp holds computed ones)
   const double *coeff_points(const CoeffDesc &c, DeviceArray<double> &tmp, hipStream_t s) const;
   int expand_kind() const { return layout_.blocked() ? QLAYOUT_BLOCKED : QLAYOUT_NATIVE; }
   void expand_compressed(DeviceArray<double> &fd, DeviceArray<double> &fm, hipStream_t s) const;

 public:
   void record_start_public(hipStream_t s) { record_start(s); }
   void record_stop_public(hipStream_t s) { record_stop(s); }

 private:
   int ne_, order_, ndofs_, n_owned_, D_, Q_, ND_, NQ_;
   DofToQuad maps_;
   Basis1D basis_, basis1_;
   QLayout layout_;
   int mode_ = KERNEL_AUTO, resolved_mode_ = KERNEL_AUTO;
   int scatter_ = SCATTER_PARTIALS;
   int n_sh_ = 0, n_sh_owned_ = 0;
   long n_slots_ = 0;
   // second-pass plan (see finish_shared, kern::sum_partials): runs [nrun + 1][12], the
   // first slots of holders beyond the fourth, blocks [nblk][2] (owned runs' blocks first)
   DeviceArray<int> sh_runs_, sh_rslots_, sh_blocks_;
   DeviceArray<int> sh_pdof_;       // plan entry -> dof (runs whose dofs are not affine read it)
   long n_runs_ = 0, n_explicit_runs_ = 0;
   int sh_nblk_owned_ = 0, sh_nblk_ = 0;
   DeviceArray<double> part_;                       // partial slots: TPE [blk][nd][64]; LINE [bricks | [e][nd]]
   bool assembled_ = false;
   DeviceArray<double> diag_cache_;  // the diagonal of assembly diag_gen_ (assemble_diagonal)
   long diag_gen_ = -1;
   long gen_ = 0;
   DeviceArray<double> ywork_;      // add_mult
   bool have_mass_ = false, have_diff_ = false;
   CoeffDesc cmass_, cdiff_;
   std::vector<int> attr_;               // element attributes (set_attributes)
   std::vector<int> marker_[2];          // per integrator kind: attribute marker (empty: none)
   bool marked_[2] = {false, false};
   std::vector<int> order_added_;        // integrator kinds in AddDomainIntegrator order (the diagonal's markers)
   DeviceArray<double> emask_[2];        // per integrator kind: element weights [ne] (marked only)
   int diag_integ_ = -1;                 // the marker diagonal: integrator whose qdata diag_w_ scales (-1: none)
   DeviceArray<double> diag_w_;          // its element weights [ne] (the second integrator's marker, at Assemble)

   std::vector<int> gmap_host_;
   DeviceArray<int> gmap_;          // native [e][nd]
   DeviceArray<int> gmap_blk_;      // blocked [blk][nd][64] (internal element order)
   DeviceArray<int> gmap_line_;     // LINE: [e][nd] dof | shared << 30 | sign << 31
   DeviceArray<int> lelem_;         // LINE: elements outside bricks
   std::vector<int> lelem_off_;     // LINE: listed elements of block b = [lelem_off_[b], lelem_off_[b+1])
   std::vector<int> splits_;        // apply_blocks range boundaries besides 0 / nblk
   int n_bricks_ = 0, brick_bz_ = 0, brick_np_ = 0;  // LINE bricks: count, 2 x 2 x bz, lattice points
   DeviceArray<int> belem_, bmap_;  // LINE bricks: [nbrick][4 bz] elements, [nbrick][np] lattice map
   DeviceArray<int> breg_;          // LINE bricks, lattice-numbered: [nbrick][8] (base, sx, sy, sz, face mask)
   DeviceArray<int> treg_;          // TPE blocks: [nblk][8] (base, sx, sy, sz, face mask, -, -, flag 1 regular / 2 lattice slots)
   bool treg_all_ = false;          // every TPE block regular: face-grouped slots only
   bool cdiag_ = false;             // snapshot forms: every element's C diagonal (axis-aligned: the diagonal flux)
   DeviceArray<int> cdflag_;        // its test's device scratch
   bool tlat_all_ = false;          // every TPE block a lattice-map block (treg flag 2)
   int n_treg_ = 0;                 // regular TPE blocks
   int n_tlat_ = 0;                 // TPE blocks with face-grouped slots but map-addressed dofs (treg flag 2)
   DeviceArray<int> lmap_;          // their block lattice maps [nblk][tpe_lattice_points] (tpe_lattice_slot order)
   int part_stride_ = 0;            // TPE partial slots per block
   int plan_kind_ = -1;             // qdata layout the TPE plan (merges, regular blocks, slots) was built for
   std::vector<int> brick_off_;     // LINE bricks of block b = [brick_off_[b], brick_off_[b+1])
   long part_line_off_ = 0;         // LINE: leftover elements' partial slots start here
   int n_left_ = 0;                 // LINE: elements outside bricks
   int line_bricks_ = -1;           // requested brick mode (set_line_bricks)
   bool affine_ = false;            // every element a parallelepiped (set_element_nodes)
   bool compress_ = true;           // set_geometry_compression
   bool tsnap_pref_ = true;         // set_coefficient_snapshot
   DeviceArray<double> tsnap_;      // coefficient snapshot T' = A + B T (local L-vector)
   int latency_from_ = -1;          // set_latency_from
   bool perm_auto_ = false;         // perm_host_ was derived (not the caller's)
   DeviceArray<int> lane_flags_;    // [blk][64] in-wave merge flags
   std::vector<int> perm_host_;     // internal position -> caller element (empty: identity)
   DeviceArray<int> pos_;           // caller element -> internal position
   DeviceArray<int> perm_dev_;      // internal position -> caller element
   DeviceArray<int> csr_off_, csr_idx_;
   DeviceArray<double> enodes_;     // [e][3][8]
   DeviceArray<double> cfit_;       // TRILINEAR from Jacobians: fitted map coefficients [e][21]
   const double *jac_ = nullptr;    // device, not owned
   DeviceArray<double> W_, rowtab_, drowtab_;
   DeviceArray<BasisDev> btab_;     // device copy of basis_ + its even/odd split (line / brick / diagonal / coefficient kernels)
   const Basis1D *btab() const { return btab_.size() ? &btab_.data()->b : nullptr; }
   DeviceArray<double> qd_diff_, qd_mass_;
   DeviceArray<double> xe_, ye_;    // unfused work E-vectors
   DeviceArray<double> ctmp_m_, ctmp_d_;

   bool timing_ = false;
   std::vector<hipEvent_t> ev_start_, ev_stop_;
   size_t ev_count_ = 0;
};

} // namespace ecm2
