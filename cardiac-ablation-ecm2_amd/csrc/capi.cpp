// capi.cpp -- extern "C" boundary (include/ecm2_pa.h).  Every entry point
// catches ecm2::Error / std::exception, records the message and returns a code.
#include "../../include/ecm2_pa.h"

#include "fe.hpp"
#include "mesh.hpp"
#include "pa_form.hpp"
#include "bricks.hpp"
#include "par_form.hpp"
#include "partition.hpp"
#include "solvers.hpp"

#include <cstring>
#include <memory>
#include <string>

struct ecm2_mesh
{
   ecm2::HexMesh m;
};
struct ecm2_h1space
{
   ecm2::H1Space s;
};
struct ecm2_pa_form
{
   ecm2::PAForm *f;
};
struct ecm2_partition
{
   ecm2::LocalPart p;
};
struct ecm2_par_form
{
   ecm2::ParPAForm *f;
};
struct ecm2_operator
{
   std::unique_ptr<ecm2::LinOp> op;
};

namespace
{
thread_local std::string g_last_error;
thread_local int g_pcg_converged = 0;  // IterativeSolver::GetConverged() of the thread's last PCG

template <typename F>
int guard(F &&fn)
{
   try
   {
      fn();
      return ECM2_OK;
   }
   catch (const ecm2::Error &e)
   {
      g_last_error = e.what();
      return e.code;
   }
   catch (const std::bad_alloc &)
   {
      g_last_error = "host out of memory";
      return ECM2_ERR_INTERNAL;
   }
   catch (const std::exception &e)
   {
      g_last_error = e.what();
      return ECM2_ERR_INTERNAL;
   }
}

#define NEED(p) ECM2_VERIFY((p) != nullptr, ecm2::ERR_ARG, "null argument: " #p)

inline hipStream_t S(void *s) { return reinterpret_cast<hipStream_t>(s); }

// ecm2_pa_form_add_integrator's (kind, data, params) -> the library's coefficient descriptor
ecm2::CoeffDesc make_coeff(int coeff_kind, const double *data, const double *params)
{
   ecm2::CoeffDesc c;
   c.kind = coeff_kind;
   if (coeff_kind == ECM2_COEFF_CONSTANT) { c.value = data ? data[0] : 1.0; }
   else if (coeff_kind == ECM2_COEFF_QUAD) { c.quad = data; }
   else if (coeff_kind == ECM2_COEFF_GRIDFUNC_AFFINE)
   {
      NEED(params);
      c.lvec = data;
      c.scale = params[0];
      c.slope = params[1];
      c.t_ref = params[2];
   }
   else if (coeff_kind == ECM2_COEFF_GRIDFUNC_PERFUSION)
   {
      NEED(params);
      c.lvec = data;
      for (int i = 0; i < 6; i++) { c.p[i] = params[i]; }
   }
   else if (coeff_kind == ECM2_COEFF_GRIDFUNC) { c.lvec = data; }
   else if (coeff_kind >= ECM2_COEFF_QUAD_VECTOR && coeff_kind <= ECM2_COEFF_QUAD_MATRIX) { c.quad = data; }
   else if (coeff_kind >= ECM2_COEFF_CONST_VECTOR && coeff_kind <= ECM2_COEFF_CONST_MATRIX)
   {
      NEED(data);
      for (int i = 0; i < c.dim(); i++) { c.cv[i] = data[i]; }
   }
   else { ECM2_VERIFY(false, ecm2::ERR_ARG, "unknown coefficient kind " << coeff_kind); }
   // (a null grid function is refused by PAForm::add_integrator unless the form has no dofs: a rank
   // with an empty local space passes an empty tensor's null data pointer)
   return c;
}
} // namespace

extern "C" {

const char *ecm2_last_error(void) { return g_last_error.c_str(); }
int ecm2_version(void) { return 100; }

int ecm2_stream_read(const double *a, long n, double *out, long nout, void *stream)
{
   return guard([&] { ecm2::kern::stream_read(n, a, out, nout, S(stream)); });
}

int ecm2_stream_copy(const double *a, double *b, long n, void *stream)
{
   return guard([&] { ecm2::kern::stream_copy(n, a, b, S(stream)); });
}

int ecm2_device_count(void)
{
   int n = 0;
   if (hipGetDeviceCount(&n) != hipSuccess) { return 0; }
   return n;
}

// ---- mesh ----
int ecm2_mesh_cartesian(int nx, int ny, int nz, double sx, double sy, double sz, ecm2_mesh **out)
{
   return guard([&] {
      NEED(out);
      *out = new ecm2_mesh{ecm2::HexMesh::cartesian(nx, ny, nz, sx, sy, sz)};
   });
}

int ecm2_mesh_cartesian_ex(int nx, int ny, int nz, double sx, double sy, double sz, int sfc_ordering,
                           ecm2_mesh **out)
{
   return guard([&] {
      NEED(out);
      *out = new ecm2_mesh{ecm2::HexMesh::cartesian(nx, ny, nz, sx, sy, sz, sfc_ordering != 0)};
   });
}

int ecm2_mesh_read(const char *path, ecm2_mesh **out)
{
   return guard([&] {
      NEED(path);
      NEED(out);
      *out = new ecm2_mesh{ecm2::HexMesh::read(path)};
   });
}

int ecm2_mesh_refine_uniform(ecm2_mesh *m)
{
   return guard([&] { NEED(m); m->m.refine_uniform(); });
}

int ecm2_mesh_info(const ecm2_mesh *m, int *nv, int *ne)
{
   return guard([&] {
      NEED(m);
      if (nv) { *nv = m->m.nv; }
      if (ne) { *ne = m->m.ne; }
   });
}

int ecm2_mesh_get_vertices(const ecm2_mesh *m, double *out)
{
   return guard([&] {
      NEED(m); NEED(out);
      std::memcpy(out, m->m.vert.data(), m->m.vert.size() * sizeof(double));
   });
}

int ecm2_mesh_set_vertices(ecm2_mesh *m, const double *in)
{
   return guard([&] {
      NEED(m); NEED(in);
      std::memcpy(m->m.vert.data(), in, m->m.vert.size() * sizeof(double));
   });
}

int ecm2_mesh_get_elements(const ecm2_mesh *m, int *out)
{
   return guard([&] {
      NEED(m); NEED(out);
      std::memcpy(out, m->m.elem.data(), m->m.elem.size() * sizeof(int));
   });
}

int ecm2_mesh_get_attributes(const ecm2_mesh *m, int *out)
{
   return guard([&] {
      NEED(m); NEED(out);
      std::memcpy(out, m->m.attr.data(), m->m.attr.size() * sizeof(int));
   });
}

int ecm2_mesh_set_attributes(ecm2_mesh *m, const int *in)
{
   return guard([&] {
      NEED(m); NEED(in);
      for (int e = 0; e < m->m.ne; e++) { ECM2_VERIFY(in[e] >= 1, ecm2::ERR_ARG, "element attributes are >= 1"); }
      m->m.attr.assign(in, in + m->m.ne);
   });
}

int ecm2_mesh_get_element_nodes(const ecm2_mesh *m, double *out)
{
   return guard([&] {
      NEED(m); NEED(out);
      std::vector<double> en;
      m->m.element_nodes(en);
      std::memcpy(out, en.data(), en.size() * sizeof(double));
   });
}

static void quad_points(const ecm2::HexMesh &m, int q1d, const int *elems, int n, double *out)
{
   ECM2_VERIFY(q1d >= 1 && q1d <= ecm2::MAX_Q1D, ecm2::ERR_ARG, "bad q1d " << q1d);
   std::vector<double> x(q1d), w(q1d);
   ecm2::gauss_legendre(q1d, x.data(), w.data());
   const int nq = q1d * q1d * q1d;
   for (int i = 0; i < n; i++)
   {
      const int e = elems ? elems[i] : i;
      ECM2_VERIFY(e >= 0 && e < m.ne, ecm2::ERR_ARG, "element index " << e << " out of range");
      double X[24];
      for (int c = 0; c < 3; c++)
         for (int a = 0; a < 8; a++) { X[c * 8 + a] = m.vert[3 * (size_t)m.elem[8 * (size_t)e + ecm2::kLexToNative[a]] + c]; }
      for (int q = 0; q < nq; q++)
      {
         const double xi[3] = {x[q % q1d], x[(q / q1d) % q1d], x[q / (q1d * q1d)]};
         for (int c = 0; c < 3; c++)
         {
            double v = 0.0;
            for (int a = 0; a < 8; a++)
            {
               const int ax = a & 1, ay = (a >> 1) & 1, az = a >> 2;
               v += (ax ? xi[0] : 1 - xi[0]) * (ay ? xi[1] : 1 - xi[1]) * (az ? xi[2] : 1 - xi[2]) * X[c * 8 + a];
            }
            out[((size_t)i * nq + q) * 3 + c] = v;
         }
      }
   }
}

int ecm2_mesh_quadrature_points(const ecm2_mesh *m, int q1d, double *out)
{
   return guard([&] { NEED(m); NEED(out); quad_points(m->m, q1d, nullptr, m->m.ne, out); });
}

int ecm2_mesh_quadrature_points_subset(const ecm2_mesh *m, int q1d, const int *elems, int n, double *out)
{
   return guard([&] { NEED(m); NEED(out); ECM2_VERIFY(n == 0 || elems, ecm2::ERR_ARG, "null elems"); quad_points(m->m, q1d, elems, n, out); });
}

int ecm2_mesh_element_order(const ecm2_mesh *m, int kind, int *perm)
{
   return guard([&] {
      NEED(m); NEED(perm);
      const std::vector<int> p = ecm2::element_order(m->m, kind);
      std::memcpy(perm, p.data(), p.size() * sizeof(int));
   });
}

void ecm2_mesh_destroy(ecm2_mesh *m) { delete m; }

// ---- space ----
int ecm2_h1space_create(const ecm2_mesh *m, int order, int numbering, ecm2_h1space **out)
{
   return guard([&] {
      NEED(m); NEED(out);
      *out = new ecm2_h1space{ecm2::H1Space::build(m->m, order, numbering)};
   });
}

int ecm2_h1space_info(const ecm2_h1space *s, int *ndofs, int *ne, int *nd)
{
   return guard([&] {
      NEED(s);
      if (ndofs) { *ndofs = s->s.ndofs; }
      if (ne) { *ne = s->s.ne; }
      if (nd) { *nd = s->s.nd; }
   });
}

int ecm2_h1space_get_gather_map(const ecm2_h1space *s, int *out)
{
   return guard([&] {
      NEED(s); NEED(out);
      std::memcpy(out, s->s.gather_map.data(), s->s.gather_map.size() * sizeof(int));
   });
}

int ecm2_h1space_element_order(const ecm2_h1space *s, int *perm)
{
   return guard([&] {
      NEED(s); NEED(perm);
      const std::vector<int> p = ecm2::face_brick_order(s->s.ne, s->s.order + 1, s->s.gather_map);
      std::memcpy(perm, p.data(), p.size() * sizeof(int));
   });
}

int ecm2_h1space_boundary_dofs(const ecm2_h1space *s, int *out, int *count)
{
   return guard([&] {
      NEED(s); NEED(count);
      const int n = (int)s->s.bdr_dofs.size();
      if (out)
      {
         ECM2_VERIFY(*count >= n, ecm2::ERR_ARG, "boundary dof buffer too small");
         std::memcpy(out, s->s.bdr_dofs.data(), n * sizeof(int));
      }
      *count = n;
   });
}

int ecm2_h1space_dof_coords(const ecm2_h1space *s, const ecm2_mesh *m, double *out)
{
   return guard([&] {
      NEED(s); NEED(m); NEED(out);
      std::vector<double> c;
      s->s.dof_coords(m->m, c);
      std::memcpy(out, c.data(), c.size() * sizeof(double));
   });
}

void ecm2_h1space_destroy(ecm2_h1space *s) { delete s; }

// ---- PA form ----
int ecm2_pa_form_create(int ne, int order, int ndofs, const int *gather_map, int q1d,
                        ecm2_pa_form **out)
{
   return guard([&] {
      NEED(out);
      *out = nullptr;
      auto *f = new ecm2::PAForm(ne, order, ndofs, gather_map, q1d);
      *out = new ecm2_pa_form{f};
   });
}

int ecm2_pa_form_set_element_nodes(ecm2_pa_form *f, const double *enodes)
{
   return guard([&] { NEED(f); f->f->set_element_nodes(enodes); });
}

int ecm2_pa_form_set_jacobians(ecm2_pa_form *f, const double *J)
{
   return guard([&] { NEED(f); f->f->set_jacobians(J); });
}

int ecm2_pa_form_add_integrator(ecm2_pa_form *f, int integrator, int coeff_kind,
                                const double *data, const double *params)
{
   return guard([&] {
      NEED(f);
      f->f->add_integrator(integrator, make_coeff(coeff_kind, data, params));
   });
}

int ecm2_pa_form_add_integrator_marked(ecm2_pa_form *f, int integrator, int coeff_kind, const double *data,
                                       const double *params, const int *marker, int n_marker)
{
   return guard([&] {
      NEED(f); NEED(marker);
      f->f->add_integrator(integrator, make_coeff(coeff_kind, data, params), marker, n_marker);
   });
}

int ecm2_pa_form_set_attributes(ecm2_pa_form *f, const int *attr)
{
   return guard([&] { NEED(f); f->f->set_attributes(attr); });
}

int ecm2_pa_form_set_element_order(ecm2_pa_form *f, const int *perm)
{
   return guard([&] { NEED(f); NEED(perm); f->f->set_element_order(perm); });
}

int ecm2_pa_form_set_kernel(ecm2_pa_form *f, int kernel)
{
   return guard([&] { NEED(f); f->f->set_kernel(kernel); });
}

int ecm2_pa_form_set_scatter(ecm2_pa_form *f, int mode)
{
   return guard([&] { NEED(f); f->f->set_scatter(mode); });
}

int ecm2_pa_form_set_geometry_compression(ecm2_pa_form *f, int on)
{
   return guard([&] { NEED(f); f->f->set_geometry_compression(on != 0); });
}

int ecm2_pa_form_set_coefficient_snapshot(ecm2_pa_form *f, int on)
{
   return guard([&] { NEED(f); f->f->set_coefficient_snapshot(on != 0); });
}

int ecm2_pa_form_coefficient_snapshot(const ecm2_pa_form *f, int *on)
{
   return guard([&] { NEED(f); NEED(on); *on = f->f->coefficient_snapshot() ? 1 : 0; });
}

int ecm2_pa_form_snapshot_info(const ecm2_pa_form *f, int *on, int *mass_values, int *law_at_point)
{
   return guard([&] {
      NEED(f);
      if (on) { *on = f->f->coefficient_snapshot() ? 1 : 0; }
      if (mass_values) { *mass_values = f->f->snapshot_mass(); }
      if (law_at_point) { *law_at_point = f->f->snapshot_law_at_point(); }
   });
}

int ecm2_pa_form_flux_diagonal(const ecm2_pa_form *f, int *on)
{
   return guard([&] { NEED(f); NEED(on); *on = f->f->flux_diagonal() ? 1 : 0; });
}

int ecm2_pa_form_energy_parts(const ecm2_pa_form *f, int *parts)
{
   return guard([&] { NEED(f); NEED(parts); *parts = f->f->energy_parts(); });
}

int ecm2_pa_form_set_bricks(ecm2_pa_form *f, int bz)
{
   return guard([&] { NEED(f); f->f->set_line_bricks(bz); });
}

int ecm2_pa_form_brick_info(const ecm2_pa_form *f, int *n_bricks, int *bz)
{
   return guard([&] {
      NEED(f);
      if (n_bricks) { *n_bricks = f->f->n_bricks(); }
      if (bz) { *bz = f->f->brick_bz(); }
   });
}

static void addressing_info(const ecm2::PAForm &f, int *lattice, int *n_units, long *n_runs)
{
   if (lattice) { *lattice = f.lattice_units(); }
   if (n_units) { *n_units = f.n_units(); }
   if (n_runs) { *n_runs = f.n_summation_runs(); }
}

int ecm2_pa_form_addressing_info(const ecm2_pa_form *f, int *lattice, int *n_units, long *n_runs)
{
   return guard([&] {
      NEED(f);
      addressing_info(*f->f, lattice, n_units, n_runs);
   });
}

int ecm2_par_form_addressing_info(const ecm2_par_form *f, int *lattice, int *n_units, long *n_runs)
{
   return guard([&] {
      NEED(f);
      addressing_info(f->f->local(), lattice, n_units, n_runs);
   });
}

int ecm2_pa_form_plan_info(const ecm2_pa_form *f, int *lattice_slot_units, long *n_explicit_runs)
{
   return guard([&] {
      NEED(f);
      if (lattice_slot_units) { *lattice_slot_units = f->f->lattice_slot_units(); }
      if (n_explicit_runs) { *n_explicit_runs = f->f->n_explicit_runs(); }
   });
}

int ecm2_pa_form_scatter_info(const ecm2_pa_form *f, int *n_shared, long *n_slots)
{
   return guard([&] {
      NEED(f);
      if (n_shared) { *n_shared = f->f->n_shared(); }
      if (n_slots) { *n_slots = f->f->n_partial_slots(); }
   });
}

int ecm2_pa_form_assemble(ecm2_pa_form *f, void *stream)
{
   return guard([&] { NEED(f); f->f->assemble(S(stream)); });
}

int ecm2_pa_form_mult(ecm2_pa_form *f, const double *x, double *y, void *stream)
{
   return guard([&] { NEED(f); f->f->mult(x, y, S(stream)); });
}

int ecm2_pa_form_mult_transpose(ecm2_pa_form *f, const double *x, double *y, void *stream)
{
   // Mass + Diffusion with scalar coefficients is symmetric: A^T x = A x
   return guard([&] { NEED(f); f->f->mult(x, y, S(stream)); });
}

int ecm2_pa_form_add_mult(ecm2_pa_form *f, const double *x, double *y, double a, void *stream)
{
   return guard([&] { NEED(f); f->f->add_mult(x, y, a, S(stream)); });
}

int ecm2_pa_form_assemble_diagonal(ecm2_pa_form *f, double *diag, void *stream)
{
   return guard([&] { NEED(f); NEED(diag); f->f->assemble_diagonal(diag, S(stream)); });
}

int ecm2_pa_form_restriction_mult(ecm2_pa_form *f, const double *x, double *xe, void *stream)
{
   return guard([&] { NEED(f); NEED(x); NEED(xe); f->f->restriction_mult(x, xe, S(stream)); });
}

int ecm2_pa_form_restriction_mult_transpose(ecm2_pa_form *f, const double *xe, double *y, void *stream)
{
   return guard([&] { NEED(f); NEED(xe); NEED(y); f->f->restriction_mult_transpose(xe, y, S(stream)); });
}

int ecm2_pa_form_integrator_add_mult(ecm2_pa_form *f, int integrator, const double *xe,
                                     double *ye, void *stream)
{
   return guard([&] {
      NEED(f); NEED(xe); NEED(ye);
      f->f->integrator_add_mult(integrator, xe, ye, S(stream));
   });
}

int ecm2_pa_form_get_qdata(ecm2_pa_form *f, int integrator, double *out, void *stream)
{
   return guard([&] { NEED(f); NEED(out); f->f->get_qdata(integrator, out, S(stream)); });
}

int ecm2_pa_form_info(const ecm2_pa_form *f, int *ne, int *ndofs, int *d1d, int *q1d,
                      int *kernel, int *layout)
{
   return guard([&] {
      NEED(f);
      if (ne) { *ne = f->f->ne(); }
      if (ndofs) { *ndofs = f->f->ndofs(); }
      if (d1d) { *d1d = f->f->d1d(); }
      if (q1d) { *q1d = f->f->q1d(); }
      if (kernel) { *kernel = f->f->kernel_mode(); }
      if (layout) { *layout = f->f->layout(); }
   });
}

int ecm2_pa_form_timing(ecm2_pa_form *f, int enable)
{
   return guard([&] { NEED(f); f->f->timing_enable(enable != 0); });
}

int ecm2_pa_form_timing_get(ecm2_pa_form *f, double *total_ms, long *launches)
{
   return guard([&] { NEED(f); f->f->timing_get(total_ms, launches); });
}

int ecm2_pa_form_algorithmic_bytes(const ecm2_pa_form *f, double *bytes)
{
   return guard([&] { NEED(f); NEED(bytes); *bytes = (double)f->f->algorithmic_bytes(); });
}

int ecm2_pa_form_qdata_bytes(const ecm2_pa_form *f, double *bytes)
{
   return guard([&] { NEED(f); NEED(bytes); *bytes = (double)f->f->qdata_bytes(); });
}

void ecm2_pa_form_destroy(ecm2_pa_form *f)
{
   if (f) { delete f->f; delete f; }
}

int ecm2_pcg_last_converged(void) { return g_pcg_converged; }

int ecm2_pcg_solve(ecm2_pa_form *f, const int *ess, int n_ess, const double *b, double *x,
                   double rel_tol, double abs_tol, int max_iter, int jacobi, int *iterations,
                   double *final_norm, void *stream)
{
   return guard([&] {
      NEED(f); NEED(b); NEED(x);
      g_pcg_converged = 0;
      ECM2_VERIFY(n_ess == 0 || ess, ecm2::ERR_ARG, "null essential dof list");
      const ecm2::PCGResult r = ecm2::pcg_solve(*f->f, ess, n_ess, b, x, rel_tol, abs_tol,
                                                max_iter, jacobi != 0, S(stream));
      if (iterations) { *iterations = r.iterations; }
      if (final_norm) { *final_norm = r.final_norm; }
      g_pcg_converged = r.converged ? 1 : 0;
   });
}

// ---- partition / distributed form ----
int ecm2_partition_slabs_z(const ecm2_mesh *m, int nranks, int *elem_rank)
{
   return guard([&] {
      NEED(m); NEED(elem_rank);
      const std::vector<int> er = ecm2::partition_slabs_z(m->m, nranks);
      std::memcpy(elem_rank, er.data(), er.size() * sizeof(int));
   });
}

int ecm2_partition_bricks(const ecm2_mesh *m, int nranks, int cell, int *elem_rank)
{
   return guard([&] {
      NEED(m); NEED(elem_rank);
      const std::vector<int> er = ecm2::partition_bricks(m->m, nranks, cell);
      std::memcpy(elem_rank, er.data(), er.size() * sizeof(int));
   });
}

int ecm2_partition_create(const ecm2_h1space *s, const ecm2_mesh *m, const int *elem_rank, int rank,
                          int nranks, ecm2_partition **out)
{
   return guard([&] {
      NEED(s); NEED(elem_rank); NEED(out);
      std::vector<int> er(elem_rank, elem_rank + s->s.ne);
      const bool cart = m && m->m.nx > 0 && m->m.ne == s->s.ne;
      *out = new ecm2_partition{ecm2::build_local_part(s->s, er, rank, nranks, cart ? &m->m : nullptr)};
   });
}

int ecm2_partition_create_ex(const ecm2_h1space *s, const ecm2_mesh *m, const int *elem_rank, int rank,
                             int nranks, int decomposition, ecm2_partition **out)
{
   return guard([&] {
      NEED(s); NEED(elem_rank); NEED(out);
      ECM2_VERIFY(decomposition == ECM2_DECOMP_RAP || decomposition == ECM2_DECOMP_OVERLAP, ecm2::ERR_ARG,
                  "unknown decomposition " << decomposition);
      std::vector<int> er(elem_rank, elem_rank + s->s.ne);
      const bool cart = m && m->m.nx > 0 && m->m.ne == s->s.ne;
      *out = new ecm2_partition{ecm2::build_local_part(s->s, er, rank, nranks, cart ? &m->m : nullptr,
                                                       decomposition == ECM2_DECOMP_OVERLAP)};
   });
}

int ecm2_partition_decomposition(const ecm2_partition *p, int *decomposition, int *ne_owned)
{
   return guard([&] {
      NEED(p);
      if (decomposition) { *decomposition = p->p.overlap ? ECM2_DECOMP_OVERLAP : ECM2_DECOMP_RAP; }
      if (ne_owned) { *ne_owned = p->p.ne_owned; }
   });
}

int ecm2_partition_info(const ecm2_partition *p, int *ne_local, int *ne_interior, int *n_owned,
                        int *n_ghost, int *n_nbrs, int *n_send)
{
   return guard([&] {
      NEED(p);
      if (ne_local) { *ne_local = p->p.ne_local; }
      if (ne_interior) { *ne_interior = p->p.ne_interior; }
      if (n_owned) { *n_owned = p->p.n_owned; }
      if (n_ghost) { *n_ghost = p->p.n_ghost; }
      if (n_nbrs) { *n_nbrs = (int)p->p.nbrs.size(); }
      if (n_send) { *n_send = (int)p->p.send_idx.size(); }
   });
}

int ecm2_partition_get(const ecm2_partition *p, int *elems, int *local_to_global, int *gather_map,
                       int *nbrs, int *send_off, int *send_idx, int *recv_off)
{
   return guard([&] {
      NEED(p);
      auto cp = [](int *dst, const std::vector<int> &v) {
         if (dst && !v.empty()) { std::memcpy(dst, v.data(), v.size() * sizeof(int)); }
      };
      cp(elems, p->p.elems);
      cp(local_to_global, p->p.local_to_global);
      cp(gather_map, p->p.gather_map);
      cp(nbrs, p->p.nbrs);
      cp(send_off, p->p.send_off);
      cp(send_idx, p->p.send_idx);
      cp(recv_off, p->p.recv_off);
   });
}

void ecm2_partition_destroy(ecm2_partition *p) { delete p; }

int ecm2_rccl_unique_id(unsigned char *id128)
{
   return guard([&] { NEED(id128); ecm2::rccl_unique_id(id128); });
}

int ecm2_par_form_create(const ecm2_partition *p, const double *enodes_local, int q1d,
                         const unsigned char *rccl_id, ecm2_par_form **out)
{
   return guard([&] {
      NEED(p); NEED(out);
      ECM2_VERIFY(p->p.ne_local == 0 || enodes_local, ecm2::ERR_ARG, "null element nodes");
      *out = nullptr;
      auto *f = new ecm2::ParPAForm(p->p, enodes_local, q1d, rccl_id);
      *out = new ecm2_par_form{f};
   });
}

int ecm2_par_form_add_integrator(ecm2_par_form *f, int integrator, int coeff_kind,
                                 const double *data, const double *params)
{
   return guard([&] {
      NEED(f);
      f->f->local().add_integrator(integrator, make_coeff(coeff_kind, data, params));
   });
}

int ecm2_par_form_add_integrator_marked(ecm2_par_form *f, int integrator, int coeff_kind, const double *data,
                                        const double *params, const int *marker, int n_marker)
{
   return guard([&] {
      NEED(f); NEED(marker);
      f->f->local().add_integrator(integrator, make_coeff(coeff_kind, data, params), marker, n_marker);
   });
}

int ecm2_par_form_set_attributes(ecm2_par_form *f, const int *attr_local)
{
   return guard([&] { NEED(f); f->f->local().set_attributes(attr_local); });
}

int ecm2_par_form_set_bricks(ecm2_par_form *f, int bz)
{
   return guard([&] { NEED(f); f->f->local().set_line_bricks(bz); });
}

int ecm2_par_form_set_schedule(ecm2_par_form *f, int schedule, int graph)
{
   return guard([&] {
      NEED(f);
      ECM2_VERIFY(schedule == ECM2_SCHEDULE_SERIAL || schedule == ECM2_SCHEDULE_OVERLAP, ecm2::ERR_ARG,
                  "schedule " << schedule << " not ECM2_SCHEDULE_SERIAL / ECM2_SCHEDULE_OVERLAP");
      f->f->set_schedule(schedule == ECM2_SCHEDULE_SERIAL, graph);
   });
}

int ecm2_par_form_set_scatter(ecm2_par_form *f, int mode)
{
   return guard([&] { NEED(f); f->f->local().set_scatter(mode); });
}

int ecm2_rccl_p2p_selftest(int graph, int n, double *max_err)
{
   return guard([&] {
      NEED(max_err);
      ECM2_VERIFY(n >= 1, ecm2::ERR_ARG, "n >= 1");
      *max_err = ecm2::rccl_p2p_selftest(graph != 0, n);
   });
}

int ecm2_par_form_set_geometry_compression(ecm2_par_form *f, int on)
{
   return guard([&] { NEED(f); f->f->local().set_geometry_compression(on != 0); });
}

int ecm2_par_form_set_kernel(ecm2_par_form *f, int kernel)
{
   return guard([&] {
      NEED(f);
      ECM2_VERIFY(kernel != ECM2_KERNEL_UNFUSED, ecm2::ERR_UNSUPPORTED, "distributed form needs a fused kernel");
      f->f->local().set_kernel(kernel);
   });
}

int ecm2_par_form_assemble(ecm2_par_form *f, void *stream)
{
   return guard([&] { NEED(f); f->f->assemble(S(stream)); });
}

int ecm2_par_form_mult(ecm2_par_form *f, const double *x_true, double *y_true, void *stream)
{
   return guard([&] {
      NEED(f);
      ECM2_VERIFY(f->f->true_size() == 0 || (x_true && y_true), ecm2::ERR_ARG, "null vector");
      f->f->mult(x_true, y_true, S(stream));
   });
}

int ecm2_par_form_mult_transpose(ecm2_par_form *f, const double *x_true, double *y_true, void *stream)
{
   // P^T A^T P = P^T A P (A symmetric)
   return ecm2_par_form_mult(f, x_true, y_true, stream);
}

int ecm2_partition_exchange_schedule(const ecm2_partition *p, int transpose, int *out, int *count)
{
   return guard([&] {
      NEED(p); NEED(count);
      const std::vector<ecm2::Xfer> sch = ecm2::exchange_schedule(p->p, transpose != 0);
      const int n = (int)sch.size();
      if (out)
      {
         ECM2_VERIFY(*count >= n, ecm2::ERR_ARG, "schedule buffer too small");
         for (int i = 0; i < n; i++)
         {
            const ecm2::Xfer &t = sch[i];
            const int row[5] = {t.peer, t.send, t.buf, t.off, t.count};
            std::memcpy(out + 5 * i, row, sizeof(row));
         }
      }
      *count = n;
   });
}

int ecm2_par_group_mult(ecm2_par_form *const *forms, int n, const double *const *x_true,
                        double *const *y_true, void *stream)
{
   return guard([&] {
      NEED(forms); NEED(x_true); NEED(y_true);
      std::vector<ecm2::ParPAForm *> fs;
      std::vector<const double *> xs;
      std::vector<double *> ys;
      for (int i = 0; i < n; i++)
      {
         NEED(forms[i]);
         fs.push_back(forms[i]->f);
         xs.push_back(x_true[i]);
         ys.push_back(y_true[i]);
      }
      ecm2::par_group_mult(fs, xs, ys, S(stream));
   });
}

int ecm2_par_group_mult_rccl(ecm2_par_form *const *forms, int n, const double *const *x_true,
                             double *const *y_true, void *stream)
{
   return guard([&] {
      NEED(forms); NEED(x_true); NEED(y_true);
      std::vector<ecm2::ParPAForm *> fs;
      std::vector<const double *> xs;
      std::vector<double *> ys;
      for (int i = 0; i < n; i++)
      {
         NEED(forms[i]);
         fs.push_back(forms[i]->f);
         xs.push_back(x_true[i]);
         ys.push_back(y_true[i]);
      }
      ecm2::par_group_mult(fs, xs, ys, S(stream), true);
   });
}

int ecm2_par_group_mult_member(ecm2_par_form *const *forms, int n, int member, const double *const *x_true,
                               double *const *y_true, void *stream)
{
   return guard([&] {
      NEED(forms); NEED(x_true); NEED(y_true);
      std::vector<ecm2::ParPAForm *> fs;
      std::vector<const double *> xs;
      std::vector<double *> ys;
      for (int i = 0; i < n; i++)
      {
         NEED(forms[i]);
         fs.push_back(forms[i]->f);
         xs.push_back(x_true[i]);
         ys.push_back(y_true[i]);
      }
      ecm2::par_group_mult_member(fs, xs, ys, member, S(stream));
   });
}

int ecm2_par_form_assemble_diagonal(ecm2_par_form *f, double *d_true, void *stream)
{
   return guard([&] { NEED(f); NEED(d_true); f->f->assemble_diagonal(d_true, S(stream)); });
}

int ecm2_par_group_diagonal(ecm2_par_form *const *forms, int n, double *const *d_true, void *stream)
{
   return guard([&] {
      NEED(forms); NEED(d_true);
      std::vector<ecm2::ParPAForm *> fs;
      std::vector<double *> ds;
      for (int i = 0; i < n; i++)
      {
         NEED(forms[i]);
         fs.push_back(forms[i]->f);
         ds.push_back(d_true[i]);
      }
      ecm2::par_group_diagonal(fs, ds, S(stream));
   });
}

// ---- operators and their solvers ----
int ecm2_operator_from_pa_form(ecm2_pa_form *f, ecm2_operator **out)
{
   return guard([&] {
      NEED(f); NEED(out);
      *out = new ecm2_operator{std::unique_ptr<ecm2::LinOp>(new ecm2::FormOp(*f->f))};
   });
}

int ecm2_operator_from_par_form(ecm2_par_form *f, ecm2_operator **out)
{
   return guard([&] {
      NEED(f); NEED(out);
      *out = new ecm2_operator{std::unique_ptr<ecm2::LinOp>(new ecm2::ParFormOp(*f->f))};
   });
}

int ecm2_operator_from_par_group(ecm2_par_form *const *forms, int n, ecm2_operator **out)
{
   return guard([&] {
      NEED(forms); NEED(out);
      ECM2_VERIFY(n > 0, ecm2::ERR_ARG, "empty group");
      std::vector<ecm2::ParPAForm *> fs;
      for (int i = 0; i < n; i++)
      {
         NEED(forms[i]);
         ECM2_VERIFY(forms[i]->f->part().rank == i && forms[i]->f->part().nranks == n, ecm2::ERR_ARG,
                     "loopback group: form " << i << " has rank " << forms[i]->f->part().rank);
         fs.push_back(forms[i]->f);
      }
      *out = new ecm2_operator{std::unique_ptr<ecm2::LinOp>(new ecm2::GroupOp(fs))};
   });
}

int ecm2_operator_from_par_member(ecm2_par_form *const *forms, int n, int member, ecm2_operator **out)
{
   return guard([&] {
      NEED(forms); NEED(out);
      ECM2_VERIFY(n > 0, ecm2::ERR_ARG, "empty group");
      std::vector<ecm2::ParPAForm *> fs;
      for (int i = 0; i < n; i++)
      {
         NEED(forms[i]);
         ECM2_VERIFY(forms[i]->f->part().rank == i && forms[i]->f->part().nranks == n, ecm2::ERR_ARG,
                     "loopback group: form " << i << " has rank " << forms[i]->f->part().rank);
         fs.push_back(forms[i]->f);
      }
      *out = new ecm2_operator{std::unique_ptr<ecm2::LinOp>(new ecm2::MemberOp(fs, member))};
   });
}

int ecm2_operator_size(const ecm2_operator *op, int *n)
{
   return guard([&] { NEED(op); NEED(n); *n = op->op->size(); });
}

int ecm2_operator_mult(ecm2_operator *op, const double *x, double *y, void *stream)
{
   return guard([&] { NEED(op); NEED(x); NEED(y); op->op->mult(x, y, S(stream)); });
}

int ecm2_operator_pcg(ecm2_operator *op, const int *ess, int n_ess, const double *b, double *x,
                      double rel_tol, double abs_tol, int max_iter, int jacobi, int *iterations,
                      double *final_norm, void *stream)
{
   return guard([&] {
      NEED(op); NEED(b); NEED(x);
      g_pcg_converged = 0;
      ECM2_VERIFY(n_ess == 0 || ess, ecm2::ERR_ARG, "null essential dof list");
      const ecm2::PCGResult r = ecm2::pcg_solve(*op->op, ess, n_ess, b, x, rel_tol, abs_tol, max_iter,
                                                jacobi != 0, S(stream));
      if (iterations) { *iterations = r.iterations; }
      if (final_norm) { *final_norm = r.final_norm; }
      g_pcg_converged = r.converged ? 1 : 0;
   });
}

double ecm2_ode_implicit_coeff(int type)
{
   try { return ecm2::ode_implicit_coeff(type); }
   catch (...) { return 0.0; }
}

int ecm2_ode_step(int type, ecm2_operator *T, ecm2_operator *K, double dt, double *u, const int *ess,
                  int n_ess, double rel_tol, int max_iter, int jacobi, int *solves, int *iterations,
                  int *converged, void *stream)
{
   return guard([&] {
      NEED(T); NEED(K); NEED(u);
      ECM2_VERIFY(n_ess == 0 || ess, ecm2::ERR_ARG, "null essential dof list");
      const ecm2::StepStats st = ecm2::ode_step(type, *T->op, *K->op, dt, u, ess, n_ess, rel_tol, max_iter,
                                                jacobi != 0, S(stream));
      if (solves) { *solves = st.solves; }
      if (converged) { *converged = st.converged ? 1 : 0; }
      if (iterations) { *iterations = st.iterations; }
   });
}

void ecm2_operator_destroy(ecm2_operator *op) { delete op; }

int ecm2_par_form_timing(ecm2_par_form *f, int enable)
{
   return guard([&] { NEED(f); f->f->local().timing_enable(enable != 0); });
}

int ecm2_par_form_timing_get(ecm2_par_form *f, double *total_ms, long *launches)
{
   return guard([&] { NEED(f); f->f->local().timing_get(total_ms, launches); });
}

int ecm2_par_form_algorithmic_bytes(const ecm2_par_form *f, double *bytes)
{
   return guard([&] {
      NEED(f); NEED(bytes);
      // local subdomain: interface dofs counted once per owner copy
      *bytes = (double)f->f->algorithmic_bytes();
   });
}

int ecm2_par_form_coefficient_snapshot(const ecm2_par_form *f, int *on)
{
   return guard([&] { NEED(f); NEED(on); *on = f->f->local().coefficient_snapshot() ? 1 : 0; });
}

int ecm2_par_form_qdata_bytes(const ecm2_par_form *f, double *bytes)
{
   return guard([&] { NEED(f); NEED(bytes); *bytes = (double)f->f->local().qdata_bytes(); });
}

int ecm2_par_form_layout(const ecm2_par_form *f, int *layout)
{
   return guard([&] { NEED(f); NEED(layout); *layout = f->f->local().layout(); });
}

int ecm2_par_form_info(const ecm2_par_form *f, int *n_true, int *kernel)
{
   return guard([&] {
      NEED(f);
      if (n_true) { *n_true = f->f->true_size(); }
      if (kernel) { *kernel = f->f->local().kernel_mode(); }
   });
}

void ecm2_par_form_destroy(ecm2_par_form *f)
{
   if (f) { delete f->f; delete f; }
}

} // extern "C"
