/*
 * ecm2_pa.h -- C ABI of the MI355X-native PA diffusion+mass operator.
 *
 * This is the drop-in boundary for the reference's
 *   BilinearForm(PARTIAL) + MassIntegrator(alpha) + DiffusionIntegrator(beta)
 * hot path (PABilinearFormExtension, fem/bilinearform_ext.hpp:67-144).  Plain C:
 * opaque handles, plain pointers and sizes, int status codes (0 = ok), no HIP or
 * torch types.  Streams are passed as `void *` holding a hipStream_t (NULL = the
 * null stream, which is what the reference uses: general/forall.hpp:782).
 *
 * Memory: arguments documented "host" are read during the call; arguments
 * documented "device" are HBM pointers (hipMalloc / torch CUDA tensors).
 * Errors mirror MFEM_VERIFY -> mfem_error (general/error.cpp:154-184): the call
 * returns a nonzero ECM2_ERR_* code and ecm2_last_error() holds the message.
 * There is no CPU fallback: without a GPU every compute entry point fails with
 * ECM2_ERR_HIP.  See INTEGRATION.md for the reference-side binding.
 */
#ifndef ECM2_PA_H
#define ECM2_PA_H

#ifdef __cplusplus
extern "C" {
#endif

#define ECM2_OK 0
#define ECM2_ERR_ARG 1
#define ECM2_ERR_HIP 2
#define ECM2_ERR_STATE 3
#define ECM2_ERR_IO 4
#define ECM2_ERR_UNSUPPORTED 5
#define ECM2_ERR_COMM 6
#define ECM2_ERR_INTERNAL 7
#define ECM2_ERR_NUMERIC 8  /* a non-finite value where the reference's MFEM_VERIFY(IsFinite(..)) aborts
                              (CGSolver::Mult's nom / den / betanom, linalg/solvers.cpp:896, 932, 954, 993) */

/* Integrator kinds (MassIntegrator, DiffusionIntegrator: fem/bilininteg.hpp:2177-2465). */
#define ECM2_MASS 0
#define ECM2_DIFFUSION 1

/* Coefficient kinds (CoefficientVector COMPRESSED storage, fem/coefficient.cpp:2006-2180). */
#define ECM2_COEFF_CONSTANT 0       /* ConstantCoefficient                                   */
#define ECM2_COEFF_QUAD 1           /* values at quadrature points, device [ne][nq]          */
#define ECM2_COEFF_GRIDFUNC_AFFINE 2/* scale*(1+slope*(T(x_q)-t_ref)), T an H1 L-vector       */
/* Pennes heat capacity + perfusion of the implicit stage's mass coefficient, T an H1 L-vector:
 *   alpha(T) = rho_c + gdt_cb * w_b(T),  w_b(T) = w0 * max(0, 1 + a (T - t0)) for T < t_stop,
 *   0 at or above t_stop (perfusion shut-down in coagulated tissue);
 * params[0..5] = (rho_c, gdt_cb, w0, a, t0, t_stop).  T is projected to the quadrature points
 * like a GridFunctionCoefficient (qfunction.cpp:73-98, coefficient.cpp:2052-2070); the law
 * itself is the bioheat application's (not in the reference snapshot: parity-unpinned). */
#define ECM2_COEFF_GRIDFUNC_PERFUSION 3
/* Vector and matrix diffusion coefficients -- anisotropic (fibre-oriented) tissue conductivity;
 * DiffusionIntegrator(VectorCoefficient | MatrixCoefficient), PADiffusionSetup3D coeffDim 3 / 6 / 9
 * (fem/integ/bilininteg_diffusion_kernels.cpp:297-348), DiffusionIntegrator only.  QUAD_*: device
 * [ne][nq][dim]; CONST_*: host data[dim].  dim 3: diag(v); 6: symmetric (11,12,13,22,23,33)
 * (SymmetricMatrixCoefficient::ProjectSymmetric); 9: general, row-major M(i,j) at 3 i + j (the
 * transposed projection of CoefficientVector::ProjectTranspose, coefficient.cpp:2093-2123).  These
 * keep the full per-point layout (BLOCKED / NATIVE: 6 symmetric entries); a general matrix keeps
 * the reference's 9-entry qdata (ECM2_QLAYOUT_NATIVE9) and runs the workgroup-per-element or
 * unfused kernels (ECM2_ERR_UNSUPPORTED for ECM2_KERNEL_TPE / _LINE). */
#define ECM2_COEFF_QUAD_VECTOR 4
#define ECM2_COEFF_QUAD_SYMMATRIX 5
#define ECM2_COEFF_QUAD_MATRIX 6
#define ECM2_COEFF_CONST_VECTOR 7
#define ECM2_COEFF_CONST_SYMMATRIX 8
#define ECM2_COEFF_CONST_MATRIX 9
/* GridFunctionCoefficient of an H1 field on the form's own space (fem/coefficient.cpp:250-253 ->
 * QuadratureFunction::ProjectGridFunction, qfunction.cpp:73-98): data = the field's device L-vector,
 * params NULL; the value at a point is the interpolated field (no law) -- e.g. ex16p's conductivity
 * kappa + alpha u formed at the dofs, examples/ex16p.cpp:450-466. */
#define ECM2_COEFF_GRIDFUNC 10

/* Kernel selection (all produce the same operator). */
#define ECM2_KERNEL_AUTO 0     /* TPE for p <= 2, LINE for p = 3..6                 */
#define ECM2_KERNEL_TPE 1      /* fused, thread per element (p = 1, 2)              */
#define ECM2_KERNEL_WPE 2      /* fused, workgroup per element (p = 1..6)           */
#define ECM2_KERNEL_UNFUSED 3  /* reference-shaped: R, per-integrator AddMultPA, R^T */
#define ECM2_KERNEL_LINE 4     /* fused, one wave per element, register lines (p <= 6) */

/* Numbering of H1 dofs. */
#define ECM2_NUMBERING_ENTITY 0     /* vertices, edges, faces, interiors (fespace.cpp:2767) */
#define ECM2_NUMBERING_STRUCTURED 1 /* lattice numbering of a Cartesian mesh               */

const char *ecm2_last_error(void);
int ecm2_version(void);
int ecm2_device_count(void);
/* Measurement helper (no reference counterpart): b[0..n) = a[0..n) with 16-byte
 * nontemporal loads/stores -- the HBM STREAM-copy rate bench.py reports beside the
 * spec peak.  n even, a and b 16-byte aligned device arrays. */
int ecm2_stream_copy(const double *a, double *b, long n, void *stream);
/* Read-only HBM stream over a[0..n) (16-byte nontemporal loads, a per-thread sum written to
 * out[0..nout)): the read bandwidth the read-dominated PA kernels are measured against. */
int ecm2_stream_read(const double *a, long n, double *out, long nout, void *stream);

/* ------------------------------------------------------------------------ */
/* Setup side: meshes and H1 spaces (the caller's Mesh / FiniteElementSpace)  */
/* ------------------------------------------------------------------------ */
typedef struct ecm2_mesh ecm2_mesh;
typedef struct ecm2_h1space ecm2_h1space;

/* Mesh::MakeCartesian3D(..., sfc_ordering = false), mesh/mesh.cpp:3683 (lexicographic element order). */
int ecm2_mesh_cartesian(int nx, int ny, int nz, double sx, double sy, double sz, ecm2_mesh **out);
/* Mesh::MakeCartesian3D(nx, ny, nz, HEXAHEDRON, sx, sy, sz, sfc_ordering) (mesh.hpp:898-904,
 * mesh.cpp:3683-3813): sfc_ordering = 1 (the reference's default) orders the elements along
 * NCMesh::GridSfcOrdering3D's generalized Hilbert curve (ncmesh.cpp:5435-5634). */
int ecm2_mesh_cartesian_ex(int nx, int ny, int nz, double sx, double sy, double sz, int sfc_ordering,
                           ecm2_mesh **out);
/* Mesh(filename): MFEM mesh v1.0 hex meshes and MFEM INLINE hex meshes
 * (mesh/mesh_readers.cpp:1356-1506; INLINE = Make3D with sfc_ordering, :1506).  Host file read. */
int ecm2_mesh_read(const char *path, ecm2_mesh **out);
/* Mesh::UniformRefinement, mesh/mesh.cpp:11403 (hex: 1 -> 8; UniformRefinement3D_base's vertex
 * and child numbering, mesh.cpp:10155-10290, 10635-10705). */
int ecm2_mesh_refine_uniform(ecm2_mesh *m);
int ecm2_mesh_info(const ecm2_mesh *m, int *nv, int *ne);
int ecm2_mesh_get_vertices(const ecm2_mesh *m, double *out /* host [nv][3] */);
int ecm2_mesh_set_vertices(ecm2_mesh *m, const double *in /* host [nv][3] */);
int ecm2_mesh_get_elements(const ecm2_mesh *m, int *out /* host [ne][8], native order */);
/* Element attributes (Mesh::GetAttribute / SetAttribute + SetAttributes, mesh.hpp), host [ne],
 * every attribute >= 1. */
int ecm2_mesh_get_attributes(const ecm2_mesh *m, int *out);
int ecm2_mesh_set_attributes(ecm2_mesh *m, const int *in);
/* Lexicographic corner coordinates, host out[ne][3][8]. */
int ecm2_mesh_get_element_nodes(const ecm2_mesh *m, double *out);
/* Physical coordinates of the Gauss-Legendre quadrature points of every element, host
 * out[ne][q1d^3][3] (q lexicographic, qx fastest): the points a FunctionCoefficient is
 * projected at (Coefficient::Project, fem/coefficient.cpp:52-70). */
int ecm2_mesh_quadrature_points(const ecm2_mesh *m, int q1d, double *out);
/* Same for a subset of elements (host elems[n]), out[n][q1d^3][3]. */
int ecm2_mesh_quadrature_points_subset(const ecm2_mesh *m, int q1d, const int *elems, int n,
                                       double *out);
/* Element order for the fused kernel: 0 native, 1 brick (Cartesian meshes: 4x4x4 bricks
 * first), 2 Morton order of centroids (any mesh).  perm host [ne]. */
int ecm2_mesh_element_order(const ecm2_mesh *m, int kind, int *perm);
void ecm2_mesh_destroy(ecm2_mesh *m);

/* H1_FECollection(order) + FiniteElementSpace: element->dof table in
 * lexicographic order (ElementRestriction gather_map, fem/restriction.cpp:26-107). */
int ecm2_h1space_create(const ecm2_mesh *m, int order, int numbering, ecm2_h1space **out);
int ecm2_h1space_info(const ecm2_h1space *s, int *ndofs, int *ne, int *nd);
int ecm2_h1space_get_gather_map(const ecm2_h1space *s, int *out /* host [ne][nd] */);
/* Essential true dofs for ess_bdr = all (GetEssentialTrueDofs): two-call pattern,
 * out may be NULL to query *count. */
/* Element order with 4x4x4 bricks of face-linked elements first (one per 64-lane wave of
 * the thread-per-element kernel), found from the element->dof map alone; any conforming
 * hex mesh (no reference counterpart: the reference applies elements independently,
 * fem/restriction.cpp:152-186).  perm host [ne]: internal position -> element.  Host only;
 * a PA form without an explicit order derives the same order at assemble. */
int ecm2_h1space_element_order(const ecm2_h1space *s, int *perm);
int ecm2_h1space_boundary_dofs(const ecm2_h1space *s, int *out, int *count);
int ecm2_h1space_dof_coords(const ecm2_h1space *s, const ecm2_mesh *m, double *out /* host [ndofs][3] */);
void ecm2_h1space_destroy(ecm2_h1space *s);

/* ------------------------------------------------------------------------ */
/* The PA form: drop-in for PABilinearFormExtension of Mass + Diffusion       */
/* ------------------------------------------------------------------------ */
typedef struct ecm2_pa_form ecm2_pa_form;

/* Replaces BilinearForm::SetAssemblyLevel(PARTIAL) + FiniteElementSpace
 * ElementRestriction construction (bilinearform.cpp:109-136, restriction.cpp:26-107).
 * gather_map: host [ne][(order+1)^3], MFEM gather_map semantics (-1-gid = minus sign).
 * q1d <= 0 selects the reference default rule (Q1D = order+2). */
int ecm2_pa_form_create(int ne, int order, int ndofs, const int *gather_map, int q1d,
                        ecm2_pa_form **out);
/* Geometry from lexicographic element corners, host [ne][3][8] (trilinear hexes). */
int ecm2_pa_form_set_element_nodes(ecm2_pa_form *f, const double *enodes);
/* Geometry from GeometricFactors::JACOBIANS (mesh.cpp:15242 layout NQ x 3 x 3 x NE),
 * device pointer, must stay valid until ecm2_pa_form_assemble returns. */
int ecm2_pa_form_set_jacobians(ecm2_pa_form *f, const double *J);
/* Quadrature-data layout (ecm2_pa_form_info's *layout).  AFFINE: when every element is
 * a parallelepiped (checked on the corners given to set_element_nodes, or on the Jacobians) and
 * the diffusion integrator is present, the p <= 2 fused kernel stores the constant element geometry
 * adj(J) adj(J)^T / det J once per element and one (W beta, W alpha det J) pair per
 * quadrature point (W beta alone without a MassIntegrator; W alpha det J alone with the coefficient
 * snapshot below): the reference's pa_data values (bilininteg_diffusion_kernels.cpp:349-362,
 * bilininteg_mass_pa.cpp:76) up to rounding, 3.3x fewer bytes at p = 2 (3.5x at p = 4,
 * AFFINE_E: element-ordered, for the p >= 3 line / brick kernels).  On by default;
 * ecm2_pa_form_set_geometry_compression(f, 0) keeps the full per-point layout. */
#define ECM2_QLAYOUT_NATIVE 0
#define ECM2_QLAYOUT_BLOCKED 1
#define ECM2_QLAYOUT_AFFINE 2
#define ECM2_QLAYOUT_AFFINE_E 3  /* the same compression for the p >= 3 line / brick kernels */
/* TRILINEAR (p <= 2, elements not all parallelepipeds, geometry from corners or from Jacobians
 * that a trilinear map produces): the element's trilinear-map coefficients once per element plus
 * one (W beta / det J, W alpha det J) pair per point; the fused kernel evaluates J and adj(J) at
 * every quadrature point (the reference's setup algebra, never stored): the AFFINE layout's bytes
 * on a general mesh.  TRILINEAR_E: the same for the p >= 3 line / brick kernels.  Every
 * compressed layout also serves a diffusion-only form (one W beta [/ det J] value per point). */
#define ECM2_QLAYOUT_TRILINEAR 4
#define ECM2_QLAYOUT_NATIVE9 5   /* [e][9][nq] general D_ij (a nonsymmetric matrix coefficient)    */
#define ECM2_QLAYOUT_TRILINEAR_E 6
int ecm2_pa_form_set_geometry_compression(ecm2_pa_form *f, int on);
/* Coefficient snapshot (p = 2, AFFINE layout, every 64-element block a lattice brick, the
 * diffusion coefficient a grid-function kind -- ECM2_COEFF_GRIDFUNC, _GRIDFUNC_AFFINE or
 * _GRIDFUNC_PERFUSION -- without an attribute marker): Assemble keeps a copy of the field at its
 * dofs (with an affine / identity law applied there) and the fused kernel interpolates it at the
 * quadrature points and applies the law there (as TransformedCoefficient::Eval, coefficient.cpp:262),
 * instead of storing W beta per point (the reference evaluates the same coefficient at the points in
 * its setup, coefficient.cpp:2052-2070): 8 B per point fewer.  A MassIntegrator with a constant
 * coefficient or a grid-function law of the SAME field (the Pennes heat capacity + perfusion
 * alpha(T)) then stores one value per element instead of W alpha det J per point: no per-point
 * stream at all.  The snapshot is taken at Assemble (the reference's assemble-time semantics).  On
 * by default; ecm2_pa_form_coefficient_snapshot reports whether the last Assemble took it. */
int ecm2_pa_form_set_coefficient_snapshot(ecm2_pa_form *f, int on);
int ecm2_pa_form_coefficient_snapshot(const ecm2_pa_form *f, int *on);
/* Introspection of the last Assemble's snapshot (no reference counterpart; any output may be NULL):
 * *on as above; *mass_values 0 = no MassIntegrator, 1 = W alpha det J stored per point, 2 = one value
 * per element (constant or same-field mass law); *law_at_point 1 = the field itself is interpolated and
 * the laws applied at the point, 0 = an affine / identity law applied to the snapshot's dofs. */
int ecm2_pa_form_snapshot_info(const ecm2_pa_form *f, int *on, int *mass_values, int *law_at_point);
/* Introspection (no reference counterpart): the number of partial sums of x^T A x the form's Mult
 * writes when ecm2_pcg_solve folds CGSolver's den = (A d, d) (solvers.cpp:993) into it -- one per
 * workgroup of the coefficient-snapshot kernel -- or 0 when the solver runs the dot pass instead. */
int ecm2_pa_form_energy_parts(const ecm2_pa_form *f, int *parts);
/* Introspection (no reference counterpart): *on = 1 when the last Assemble found every element's
 * adj(J) adj(J)^T / det J diagonal (axis-aligned hexahedra) and the apply kernel uses it as a diagonal -- the
 * coefficient-snapshot kernel (p = 2) or the brick kernel (AFFINE_E, p >= 3) -- with the general product's
 * values, whose off-diagonal terms would add exact zeros. */
int ecm2_pa_form_flux_diagonal(const ecm2_pa_form *f, int *on);
/* BilinearForm::AddDomainIntegrator(new MassIntegrator(Q)) / DiffusionIntegrator(Q)
 * (bilinearform.cpp:231-242).  data: CONSTANT -> data[0] (host);
 * QUAD -> device [ne][nq]; GRIDFUNC_AFFINE -> device L-vector T with
 * params[0..2] = (scale, slope, t_ref).  Device arrays must stay valid until assemble. */
int ecm2_pa_form_add_integrator(ecm2_pa_form *f, int integrator, int coeff_kind,
                                const double *data, const double *params);
/* BilinearForm::AddDomainIntegrator(integ, elem_marker) (bilinearform.cpp:237-242): as
 * ecm2_pa_form_add_integrator, restricted to the elements whose attribute a has
 * marker[a - 1] != 0 (host marker[n_marker]; the reference's PABilinearFormExtension::
 * AddMultWithMarkers, bilinearform_ext.cpp:753-774,807-847, masks the integrator's E-vector
 * output; here its quadrature data is zeroed on the excluded elements at assemble: the same
 * operator, no extra pass per Mult).  Needs ecm2_pa_form_set_attributes before assemble. */
int ecm2_pa_form_add_integrator_marked(ecm2_pa_form *f, int integrator, int coeff_kind, const double *data,
                                       const double *params, const int *marker, int n_marker);
/* Element attributes of the form's elements (the mesh's, host [ne], caller element order). */
int ecm2_pa_form_set_attributes(ecm2_pa_form *f, const int *attr);
int ecm2_pa_form_set_kernel(ecm2_pa_form *f, int kernel);
/* Scatter of the fused thread-per-element kernel (no reference counterpart: the
 * reference's ElementRestriction::MultTranspose, restriction.cpp:146-186, is the
 * deterministic CSR sum this replaces).  ECM2_SCATTER_PARTIALS (default): dofs held by
 * one element entry are stored directly, shared ones summed from per-entry partial
 * slots in a fixed order -- bitwise reproducible; ECM2_SCATTER_ATOMIC: FP64 atomics. */
#define ECM2_SCATTER_PARTIALS 0
#define ECM2_SCATTER_ATOMIC 1
int ecm2_pa_form_set_scatter(ecm2_pa_form *f, int mode);
/* Work grouping of the p >= 3 line-kernel family (no reference counterpart; the
 * reference applies each element independently, bilininteg_diffusion_kernels.hpp:989-1214):
 * bz = -1 default (2 x 2 x 1), 0 = per-element line kernel only, 1 = bricks of 2 x 2 x 1
 * elements, 2 = 2 x 2 x 2 (p = 3..6 with the default rule).  A brick is one workgroup; its
 * internal shared faces are summed in LDS in a fixed order (deterministic).  Bricks exist only
 * with ECM2_SCATTER_PARTIALS and both integrators; elements outside bricks use the line
 * kernel. */
int ecm2_pa_form_set_bricks(ecm2_pa_form *f, int bz);
/* After assemble: bricks formed and their depth (0 = none). */
int ecm2_pa_form_brick_info(const ecm2_pa_form *f, int *n_bricks, int *bz);
/* Scatter statistics after assemble: shared dofs and their partial slots. */
int ecm2_pa_form_scatter_info(const ecm2_pa_form *f, int *n_shared, long *n_slots);
/* After assemble: of the fused kernel's n_units units (p <= 2: 64-element blocks, p >= 3:
 * bricks), the `lattice` ones address their dofs arithmetically (a lattice-numbered region:
 * d = base + X sx + Y sy + Z sz with face-determined sharing, checked against the gather map;
 * the others read the map); n_runs = runs of the run-compressed summation plan.  The
 * operator is the same either way. */
int ecm2_pa_form_addressing_info(const ecm2_pa_form *f, int *lattice, int *n_units, long *n_runs);
/* Summation-plan details (introspection): units whose partial slots are face-grouped although
 * their dofs are read from the map (non-lattice numberings, e.g. the reference's entity
 * numbering), and runs whose dofs come from the plan's entry list. */
int ecm2_pa_form_plan_info(const ecm2_pa_form *f, int *lattice_slot_units, long *n_explicit_runs);
/* Optional element permutation for the fused kernel's blocked layout (host perm[ne]:
 * internal position i <- caller element perm[i]); see ecm2_mesh_element_order.  All
 * entry points keep the caller's element order (the reference's E-vector order,
 * restriction.cpp:26-107, is never exposed differently). */
int ecm2_pa_form_set_element_order(ecm2_pa_form *f, const int *perm);
/* BilinearForm::Assemble -> PABilinearFormExtension::Assemble -> AssemblePA
 * (bilinearform.cpp:456-460, bilinearform_ext.cpp:332-368). */
int ecm2_pa_form_assemble(ecm2_pa_form *f, void *stream);
/* BilinearForm::Mult / PABilinearFormExtension::Mult (bilinearform.cpp:1244-1254,
 * bilinearform_ext.cpp:487-564): y = A x, y overwritten.  x, y device [ndofs]. */
int ecm2_pa_form_mult(ecm2_pa_form *f, const double *x, double *y, void *stream);
/* PABilinearFormExtension::MultTranspose (bilinearform_ext.hpp:99, bilinearform_ext.cpp:
 * 679-): y = A^T x.  Mass + Diffusion with scalar coefficients are symmetric, so this is
 * the Mult (tests/test_gpu_parity.py asserts the equality). */
int ecm2_pa_form_mult_transpose(ecm2_pa_form *f, const double *x, double *y, void *stream);
/* Operator::AddMult (linalg/operator.hpp:108-109): y += a A x. */
int ecm2_pa_form_add_mult(ecm2_pa_form *f, const double *x, double *y, double a, void *stream);
/* PABilinearFormExtension::AssembleDiagonal (bilinearform_ext.cpp:370-454). diag device [ndofs]. */
int ecm2_pa_form_assemble_diagonal(ecm2_pa_form *f, double *diag, void *stream);
/* ElementRestriction::Mult / MultTranspose (restriction.cpp:109-186). xe device [ne][nd]. */
int ecm2_pa_form_restriction_mult(ecm2_pa_form *f, const double *x, double *xe, void *stream);
int ecm2_pa_form_restriction_mult_transpose(ecm2_pa_form *f, const double *xe, double *y, void *stream);
/* BilinearFormIntegrator::AddMultPA (bilininteg.hpp:49-97): ye += A_integ xe (E-vectors). */
int ecm2_pa_form_integrator_add_mult(ecm2_pa_form *f, int integrator, const double *xe,
                                     double *ye, void *stream);
/* pa_data in the reference layout (diffusion [ne][6][nq], mass [ne][nq]), host out. */
int ecm2_pa_form_get_qdata(ecm2_pa_form *f, int integrator, double *out, void *stream);
int ecm2_pa_form_info(const ecm2_pa_form *f, int *ne, int *ndofs, int *d1d, int *q1d,
                      int *kernel, int *layout);
/* HIP-event timing of the dominant apply kernel(s) inside Mult. */
int ecm2_pa_form_timing(ecm2_pa_form *f, int enable);
int ecm2_pa_form_timing_get(ecm2_pa_form *f, double *total_ms, long *launches);
/* SURVEY §8(d) algorithmic bytes per Mult: 8*NE*NQ*(6+1) + 16*ndofs + 4*NE*ND. */
int ecm2_pa_form_algorithmic_bytes(const ecm2_pa_form *f, double *bytes);
/* Bytes of quadrature data the form stores after assemble (diffusion + mass). */
int ecm2_pa_form_qdata_bytes(const ecm2_pa_form *f, double *bytes);
/* ~PABilinearFormExtension / BilinearForm::Update (bilinearform_ext.hpp:67-144). */
void ecm2_pa_form_destroy(ecm2_pa_form *f);

/* ------------------------------------------------------------------------ */
/* Caller: constrained Jacobi-PCG (ConstrainedOperator operator.cpp:586-646 + */
/* CGSolver::Mult solvers.cpp:869-1004)                                       */
/* ------------------------------------------------------------------------ */
/* ess: device int [n_ess] essential dofs (DIAG_ONE).  b, x device [ndofs];
 * x is overwritten (iterative_mode = false).  jacobi != 0 -> OperatorJacobiSmoother.
 * iterations = CGSolver's final_iter, final_norm = sqrt((B r, r)) (the raw (B r, r) when it is
 * negative).  CGSolver's stops: converged, max_iter, (B r, r) < 0 or (A d, d) == 0 (not
 * converged: ecm2_pcg_last_converged() == 0); a non-finite (B r, r) or (A d, d), where the
 * reference's MFEM_VERIFY aborts, returns ECM2_ERR_NUMERIC. */
int ecm2_pcg_solve(ecm2_pa_form *f, const int *ess, int n_ess, const double *b, double *x,
                   double rel_tol, double abs_tol, int max_iter, int jacobi, int *iterations,
                   double *final_norm, void *stream);
/* IterativeSolver::GetConverged() (solvers.hpp:155) of the calling thread's last
 * ecm2_pcg_solve / ecm2_operator_pcg: 1 converged, 0 not (or no solve yet). */
int ecm2_pcg_last_converged(void);

/* ------------------------------------------------------------------------ */
/* Operators for the solvers: the serial form, one rank of the RCCL form, or */
/* the in-process loopback group (concatenated true vectors), all seen as the */
/* reference's Operator (linalg/operator.hpp:24-110) by PCG and the ODE step. */
/* ------------------------------------------------------------------------ */
typedef struct ecm2_operator ecm2_operator;
typedef struct ecm2_par_form ecm2_par_form;
/* The operator keeps a reference to the form(s): destroy it first. */
int ecm2_operator_from_pa_form(ecm2_pa_form *f, ecm2_operator **out);
int ecm2_operator_from_par_form(ecm2_par_form *f, ecm2_operator **out);
/* forms[r] must be rank r of an n-rank partition; vectors are the concatenation of the
 * ranks' true vectors (rank r at offset sum_{q<r} n_owned(q)). */
int ecm2_operator_from_par_group(ecm2_par_form *const *forms, int n, ecm2_operator **out);
/* Measurement (no reference counterpart): member `member` of the loopback group as one rank's
 * operator on its own GPU -- Mult = ecm2_par_group_mult_member (the peers' x held at zero in a
 * private buffer), dots summed by ncclAllReduce on a one-rank communicator.  Vectors are the
 * member's true dofs; ecm2_operator_pcg on it times one rank's solver iteration.  OVERLAP
 * decomposition with contiguous sends (slabs) only: ECM2_ERR_UNSUPPORTED otherwise. */
int ecm2_operator_from_par_member(ecm2_par_form *const *forms, int n, int member, ecm2_operator **out);
/* Operator::Height/Width and Operator::Mult (operator.hpp:24-110). */
int ecm2_operator_size(const ecm2_operator *op, int *n);
int ecm2_operator_mult(ecm2_operator *op, const double *x, double *y, void *stream);
/* ConstrainedOperator (operator.cpp:586-646) + CGSolver::Mult (solvers.cpp:869-1004) +
 * OperatorJacobiSmoother on any operator; with the RCCL form every rank calls it
 * collectively (dots are summed with ncclAllReduce, as the reference's parallel
 * InnerProduct sums with MPI_Allreduce). */
int ecm2_operator_pcg(ecm2_operator *op, const int *ess, int n_ess, const double *b, double *x,
                      double rel_tol, double abs_tol, int max_iter, int jacobi, int *iterations,
                      double *final_norm, void *stream);
/* ODESolver::SelectImplicit types (ode.cpp:77-91): 21 BackwardEuler, 22 SDIRK23 (L-stable),
 * 23 SDIRK33, 32 ImplicitMidpoint, 33 SDIRK23 (A-stable), 34 SDIRK34.  Returns the stage
 * coefficient c (every stage solves (M + c*dt*K) k = -K u_stage), 0 for unknown types. */
double ecm2_ode_implicit_coeff(int type);
/* One step of M du/dt = -K u (ex16 ConductionOperator::ImplicitSolve, ex16.cpp:327-354, in
 * the slope form; the SDIRK stage algebra of ode.cpp:682-859).  T must be assembled as
 * M + c*dt*K with c = ecm2_ode_implicit_coeff(type); u (device, true dofs) is advanced in
 * place; ess dofs keep their values.  Stage solves: constrained Jacobi-PCG (rel_tol,
 * max_iter).  *converged = 0 if some stage solve stopped at max_iter (like CGSolver, not an
 * error). */
int ecm2_ode_step(int type, ecm2_operator *T, ecm2_operator *K, double dt, double *u, const int *ess,
                  int n_ess, double rel_tol, int max_iter, int jacobi, int *solves, int *iterations,
                  int *converged, void *stream);
void ecm2_operator_destroy(ecm2_operator *op);

/* ------------------------------------------------------------------------ */
/* Distributed form: ParBilinearForm / RAPOperator(P, A, P) over RCCL          */
/* ------------------------------------------------------------------------ */
typedef struct ecm2_partition ecm2_partition;

/* Mesh::CartesianPartitioning along z (mesh/mesh.cpp:8966) of a lexicographic Cartesian
 * mesh: elem_rank host [ne]. */
int ecm2_partition_slabs_z(const ecm2_mesh *m, int nranks, int *elem_rank);
/* Not a reference interface (the reference partitions with METIS or CartesianPartitioning):
 * equal runs of whole cell^3 element bricks of a Cartesian mesh in lexicographic brick order,
 * so that an owned-elements (ECM2_DECOMP_RAP) rank holds only whole bricks of the fused
 * kernels' blocks (balanced to one brick; measured against z-slabs in DESIGN.md §6).
 * elem_rank host [ne]. */
int ecm2_partition_bricks(const ecm2_mesh *m, int nranks, int cell, int *elem_rank);
/* Per-rank local space of a global H1 space and an element partition (ParMesh +
 * ParFiniteElementSpace, pmesh.hpp:33, pfespace.cpp:1389-1418): local L-vector
 * [owned | ghost], owner = lowest touching rank, local elements [interior | boundary],
 * neighbour exchange lists in the DeviceConformingProlongationOperator sense.  m (may be
 * NULL): when it is a Cartesian mesh the local element groups are put in brick order. */
int ecm2_partition_create(const ecm2_h1space *s, const ecm2_mesh *m, const int *elem_rank, int rank,
                          int nranks, ecm2_partition **out);
/* As ecm2_partition_create with a choice of decomposition: ECM2_DECOMP_RAP (the
 * reference's: local elements = owned elements, Mult = P, local PA, P^T) or
 * ECM2_DECOMP_OVERLAP (local elements = owned elements + every element touching an owned
 * dof, Mult = P, local PA; no P^T -- one exchange per Mult instead of two, the ghost
 * elements' outputs to non-owned dofs discarded; same operator). */
#define ECM2_DECOMP_RAP 0
#define ECM2_DECOMP_OVERLAP 1
int ecm2_partition_create_ex(const ecm2_h1space *s, const ecm2_mesh *m, const int *elem_rank, int rank,
                             int nranks, int decomposition, ecm2_partition **out);
/* Decomposition and the number of elements the rank owns (ne_local minus ghost elements). */
int ecm2_partition_decomposition(const ecm2_partition *p, int *decomposition, int *ne_owned);
int ecm2_partition_info(const ecm2_partition *p, int *ne_local, int *ne_interior, int *n_owned,
                        int *n_ghost, int *n_nbrs, int *n_send);
/* Any output may be NULL. elems [ne_local] (global ids, local order), local_to_global
 * [n_owned+n_ghost], gather_map [ne_local][nd] (local), nbrs [n_nbrs], send_off / recv_off
 * [n_nbrs+1], send_idx [n_send] (owned local indices). */
int ecm2_partition_get(const ecm2_partition *p, int *elems, int *local_to_global, int *gather_map,
                       int *nbrs, int *send_off, int *send_idx, int *recv_off);
/* The exchange schedule both transports consume (no reference counterpart; the reference's
 * per-neighbour MPI_Isend/Irecv of DeviceConformingProlongationOperator, pfespace.cpp:
 * 5394-5440 / 5496-5532, in one list): transpose = 0 for P (owners -> ghost copies), 1 for
 * P^T.  Rows of 5 ints (peer, send, buffer, offset, count), buffer 0 = the true vector x,
 * 1 = the packed send buffer [n_send], 2 = the ghost block of x [n_ghost], 3 = the ghost
 * block of y, 4 = the P^T receive buffer [n_send].  Two-call pattern: out may be NULL to
 * query *count.  Host only. */
int ecm2_partition_exchange_schedule(const ecm2_partition *p, int transpose, int *out, int *count);
/* ~ParFiniteElementSpace / ~ParMesh of the local view. */
void ecm2_partition_destroy(ecm2_partition *p);

/* ncclGetUniqueId (128 bytes) for ecm2_par_form_create; broadcast it to all ranks (the
 * reference's communicator is the ParMesh's MPI_Comm, pmesh.hpp:33). */
int ecm2_rccl_unique_id(unsigned char *id128);
/* Transport self-test (no reference counterpart): a one-rank communicator sends n doubles to
 * itself with grouped ncclSend/ncclRecv, directly (graph = 0) or captured in a HIP graph and
 * replayed (graph = 1, what ecm2_par_form_mult does); *max_err = max |received - sent|. */
int ecm2_rccl_p2p_selftest(int graph, int n, double *max_err);
/* ParBilinearForm(pfes) + SetAssemblyLevel(PARTIAL) (pbilinearform.hpp, bilinearform.cpp:
 * 109-136) on the rank's local space.  enodes_local: host [ne_local][3][8] in the
 * partition's local element order.
 * rccl_id: 128-byte id (one process per GPU, ncclCommInitRank) or NULL for a member of an
 * in-process loopback group (ecm2_par_group_mult). */
int ecm2_par_form_create(const ecm2_partition *p, const double *enodes_local, int q1d,
                         const unsigned char *rccl_id, ecm2_par_form **out);
/* As ecm2_pa_form_add_integrator, on local data: QUAD -> device [ne_local][nq] in local
 * element order; GRIDFUNC_AFFINE -> device local L-vector [n_owned + n_ghost]. */
int ecm2_par_form_add_integrator(ecm2_par_form *f, int integrator, int coeff_kind,
                                 const double *data, const double *params);
/* As ecm2_pa_form_add_integrator_marked / ecm2_pa_form_set_attributes on the local elements
 * (attributes host [ne_local], the partition's local element order). */
int ecm2_par_form_add_integrator_marked(ecm2_par_form *f, int integrator, int coeff_kind, const double *data,
                                        const double *params, const int *marker, int n_marker);
int ecm2_par_form_set_attributes(ecm2_par_form *f, const int *attr_local);
/* As ecm2_pa_form_set_kernel (fused kernels only). */
int ecm2_par_form_set_kernel(ecm2_par_form *f, int kernel);
/* Brick mode of the local form (see ecm2_pa_form_set_bricks). */
int ecm2_par_form_set_bricks(ecm2_par_form *f, int bz);
/* Schedule of the distributed Mult (no reference counterpart; the reference overlaps its
 * MPI exchange with nothing, pfespace.cpp:5394-5532): ECM2_SCHEDULE_SERIAL (default) = the P
 * exchange, ONE apply launch over every local element, the shared-dof sums, all on the
 * caller's stream; ECM2_SCHEDULE_OVERLAP = interior elements on the caller's stream beside the
 * exchange + boundary elements on a high-priority comm stream.  graph: 1 = replay one captured
 * HIP graph per (x, y), 0 = direct launches, -1 = the schedule's default (serial: direct,
 * overlap: graph).  Before Assemble. */
#define ECM2_SCHEDULE_SERIAL 0
#define ECM2_SCHEDULE_OVERLAP 1
int ecm2_par_form_set_schedule(ecm2_par_form *f, int schedule, int graph);
/* Scatter mode of the local form (ECM2_SCATTER_*; see ecm2_pa_form_set_scatter). */
int ecm2_par_form_set_scatter(ecm2_par_form *f, int mode);
/* Geometry compression of the local form (see ecm2_pa_form_set_geometry_compression). */
int ecm2_par_form_set_geometry_compression(ecm2_par_form *f, int on);
/* ParBilinearForm::Assemble -> local PABilinearFormExtension::Assemble
 * (pbilinearform.cpp:475-511, bilinearform_ext.cpp:332-368). */
int ecm2_par_form_assemble(ecm2_par_form *f, void *stream);
/* RAPOperator::Mult (operator.hpp:977): y_true = P^T A P x_true; x_true, y_true device
 * [n_owned].  Grouped ncclSend/ncclRecv, then the local PA apply and the shared-dof sums on
 * `stream` (ECM2_SCHEDULE_SERIAL, the default); see ecm2_par_form_set_schedule. */
int ecm2_par_form_mult(ecm2_par_form *f, const double *x_true, double *y_true, void *stream);
/* RAPOperator::MultTranspose (operator.hpp:979): P^T A^T P = P^T A P (A symmetric). */
int ecm2_par_form_mult_transpose(ecm2_par_form *f, const double *x_true, double *y_true, void *stream);
/* ecm2_pa_form_addressing_info for the rank's local form (its interior blocks can be
 * lattice-addressed, those touching ghost dofs are not). */
int ecm2_par_form_addressing_info(const ecm2_par_form *f, int *lattice, int *n_units, long *n_runs);
/* All subdomains of one partition in this process on one GPU (exchange by device copies that
 * follow the members' exchange schedules). */
int ecm2_par_group_mult(ecm2_par_form *const *forms, int n, const double *const *x_true,
                        double *const *y_true, void *stream);
/* Transport test (no reference counterpart): ecm2_par_group_mult with every exchange row
 * issued through RCCL -- a one-rank communicator (created on the first call, which must not be
 * inside a stream capture) ncclSend's each peer's send row to itself and ncclRecv's it into
 * the matching receive row, grouped, on `stream` (capturable).  Exercises the row buffers,
 * offsets and counts of ecm2_par_form_mult's grouped exchange on one GPU.  Serial schedule. */
int ecm2_par_group_mult_rccl(ecm2_par_form *const *forms, int n, const double *const *x_true,
                             double *const *y_true, void *stream);
/* One member's rows of the loopback group's operator (measurement of a rank's Mult on its own
 * GPU; no reference counterpart): y_true[member] = (A x)[member's true dofs], running exactly
 * the stages one RCCL rank runs (interior elements on `stream`, the P exchange -- here device
 * copies from the peers' x -- and the boundary elements on the member's comm stream, then the
 * shared-dof sums); the other members' y are not written.  Packed sends (non-slab partitions)
 * and, with RAP (serial schedule), the P^T receive copy the peers' buffers as their last
 * ecm2_par_group_mult left them (run one group Mult on the same x first).
 * ECM2_ERR_UNSUPPORTED otherwise (RAP with the overlapped schedule). */
int ecm2_par_group_mult_member(ecm2_par_form *const *forms, int n, int member, const double *const *x_true,
                               double *const *y_true, void *stream);
/* ParBilinearForm::AssembleDiagonal on the true dofs (local PA diagonal + P^T). */
int ecm2_par_form_assemble_diagonal(ecm2_par_form *f, double *d_true, void *stream);
int ecm2_par_group_diagonal(ecm2_par_form *const *forms, int n, double *const *d_true, void *stream);
/* Measurement and introspection (no reference counterpart): HIP-event timing of the local
 * apply kernels, SURVEY §8(d) bytes of the local form, true size and resolved kernel. */
int ecm2_par_form_timing(ecm2_par_form *f, int enable);
int ecm2_par_form_timing_get(ecm2_par_form *f, double *total_ms, long *launches);
int ecm2_par_form_algorithmic_bytes(const ecm2_par_form *f, double *bytes);
int ecm2_par_form_qdata_bytes(const ecm2_par_form *f, double *bytes);
/* Whether the local form's last Assemble took the coefficient snapshot
 * (ecm2_pa_form_coefficient_snapshot). */
int ecm2_par_form_coefficient_snapshot(const ecm2_par_form *f, int *on);
/* Quadrature-data layout of the local form (ECM2_QLAYOUT_*), after assemble. */
int ecm2_par_form_layout(const ecm2_par_form *f, int *layout);
int ecm2_par_form_info(const ecm2_par_form *f, int *n_true, int *kernel);
/* ~ParBilinearForm. */
void ecm2_par_form_destroy(ecm2_par_form *f);

#ifdef __cplusplus
}
#endif
#endif /* ECM2_PA_H */
