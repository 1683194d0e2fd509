// capi.cpp -- extern "C" boundary (include/ecm2_pa.h).  Every entry point
// catches ecm2::Error / std::exception, records the message and returns a code.
#include "../../include/ecm2_pa.h"

#include "fe.hpp"
#include "mesh.hpp"
#include "pa_form.hpp"

#include <cstring>
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

namespace
{
thread_local std::string g_last_error;

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
} // namespace

extern "C" {

const char *ecm2_last_error(void) { return g_last_error.c_str(); }
int ecm2_version(void) { return 100; }

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

int ecm2_mesh_get_element_nodes(const ecm2_mesh *m, double *out)
{
   return guard([&] {
      NEED(m); NEED(out);
      std::vector<double> en;
      m->m.element_nodes(en);
      std::memcpy(out, en.data(), en.size() * sizeof(double));
   });
}

int ecm2_mesh_quadrature_points(const ecm2_mesh *m, int q1d, double *out)
{
   return guard([&] {
      NEED(m); NEED(out);
      ECM2_VERIFY(q1d >= 1 && q1d <= ecm2::MAX_Q1D, ecm2::ERR_ARG, "bad q1d " << q1d);
      std::vector<double> x(q1d), w(q1d), en;
      ecm2::gauss_legendre(q1d, x.data(), w.data());
      m->m.element_nodes(en);
      const int nq = q1d * q1d * q1d;
      for (int e = 0; e < m->m.ne; e++)
         for (int q = 0; q < nq; q++)
         {
            const double xi[3] = {x[q % q1d], x[(q / q1d) % q1d], x[q / (q1d * q1d)]};
            for (int c = 0; c < 3; c++)
            {
               double v = 0.0;
               for (int a = 0; a < 8; a++)
               {
                  const int ax = a & 1, ay = (a >> 1) & 1, az = a >> 2;
                  v += (ax ? xi[0] : 1 - xi[0]) * (ay ? xi[1] : 1 - xi[1]) *
                       (az ? xi[2] : 1 - xi[2]) * en[(size_t)e * 24 + c * 8 + a];
               }
               out[((size_t)e * nq + q) * 3 + c] = v;
            }
         }
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
      ecm2::CoeffDesc c;
      c.kind = coeff_kind;
      if (coeff_kind == ECM2_COEFF_CONSTANT)
      {
         c.value = data ? data[0] : 1.0;
      }
      else if (coeff_kind == ECM2_COEFF_QUAD)
      {
         c.quad = data;
      }
      else if (coeff_kind == ECM2_COEFF_GRIDFUNC_AFFINE)
      {
         NEED(params);
         c.lvec = data;
         c.scale = params[0];
         c.slope = params[1];
         c.t_ref = params[2];
      }
      f->f->add_integrator(integrator, c);
   });
}

int ecm2_pa_form_set_kernel(ecm2_pa_form *f, int kernel)
{
   return guard([&] { NEED(f); f->f->set_kernel(kernel); });
}

int ecm2_pa_form_assemble(ecm2_pa_form *f, void *stream)
{
   return guard([&] { NEED(f); f->f->assemble(S(stream)); });
}

int ecm2_pa_form_mult(ecm2_pa_form *f, const double *x, double *y, void *stream)
{
   return guard([&] { NEED(f); f->f->mult(x, y, S(stream)); });
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

void ecm2_pa_form_destroy(ecm2_pa_form *f)
{
   if (f) { delete f->f; delete f; }
}

int ecm2_pcg_solve(ecm2_pa_form *f, const int *ess, int n_ess, const double *b, double *x,
                   double rel_tol, double abs_tol, int max_iter, int jacobi, int *iterations,
                   double *final_norm, void *stream)
{
   return guard([&] {
      NEED(f); NEED(b); NEED(x);
      ECM2_VERIFY(n_ess == 0 || ess, ecm2::ERR_ARG, "null essential dof list");
      const ecm2::PCGResult r = ecm2::pcg_solve(*f->f, ess, n_ess, b, x, rel_tol, abs_tol,
                                                max_iter, jacobi != 0, S(stream));
      if (iterations) { *iterations = r.iterations; }
      if (final_norm) { *final_norm = r.final_norm; }
   });
}

} // extern "C"
