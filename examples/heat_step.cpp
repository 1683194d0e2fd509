// heat_step.cpp -- the serial heat step of examples/ex16p.cpp (ConductionOperator with
// MassIntegrator + DiffusionIntegrator(GridFunctionCoefficient(kappa + alpha u)) at
// AssemblyLevel::PARTIAL, SetParameters after every step, an SDIRK implicit solve by
// constrained Jacobi-PCG), written against the C ABI alone (include/ecm2_pa.h) the way a C++
// host binding of the reference would call it: no Python, no torch; HIP only for device
// buffers.  Checks the known answers of the reference's own fichera fixture (1^T M 1 = |fichera|
// = 7, K 1 = 0) and that the temperature decays and stays bounded.  Exit status 0 = pass.
//
// Usage: heat_step [mesh = tests/golden/fichera.mesh] [refinements = 2] [order = 2] [steps = 5]
#include "ecm2_pa.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CHECK(call)                                                                       \
   do {                                                                                   \
      const int rc_ = (call);                                                             \
      if (rc_ != ECM2_OK)                                                                 \
      {                                                                                   \
         std::fprintf(stderr, "%s failed (%d): %s\n", #call, rc_, ecm2_last_error());     \
         std::exit(2);                                                                    \
      }                                                                                   \
   } while (0)
#define HIPCHECK(call)                                                                    \
   do {                                                                                   \
      if ((call) != hipSuccess) { std::fprintf(stderr, "%s failed\n", #call); std::exit(2); } \
   } while (0)

template <typename T>
static T *device_copy(const std::vector<T> &h)
{
   T *d = nullptr;
   HIPCHECK(hipMalloc(&d, std::max<size_t>(1, h.size()) * sizeof(T)));
   if (!h.empty()) { HIPCHECK(hipMemcpy(d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice)); }
   return d;
}

static std::vector<double> host_copy(const double *d, int n)
{
   std::vector<double> h(n);
   HIPCHECK(hipMemcpy(h.data(), d, n * sizeof(double), hipMemcpyDeviceToHost));
   return h;
}

// one PA form over the space: Mass(alpha) [+ Diffusion(scale k(T))], geometry from the corners
static ecm2_pa_form *make_form(int ne, int order, int ndofs, const std::vector<int> &gmap,
                               const std::vector<double> &enodes, double alpha, bool diffusion,
                               const double *T_dev, double kscale)
{
   ecm2_pa_form *f = nullptr;
   CHECK(ecm2_pa_form_create(ne, order, ndofs, gmap.data(), 0, &f));
   CHECK(ecm2_pa_form_set_element_nodes(f, enodes.data()));
   if (alpha != 0.0) { CHECK(ecm2_pa_form_add_integrator(f, ECM2_MASS, ECM2_COEFF_CONSTANT, &alpha, nullptr)); }
   if (diffusion)
   {
      // k(T) = k0 (1 + 0.0012 (T - 37)), the Pennes conductivity law of the bench
      const double params[3] = {kscale, 0.0012, 37.0};
      CHECK(ecm2_pa_form_add_integrator(f, ECM2_DIFFUSION, ECM2_COEFF_GRIDFUNC_AFFINE, T_dev, params));
   }
   CHECK(ecm2_pa_form_assemble(f, nullptr));
   return f;
}

// ex16p's K(u) = DiffusionIntegrator(GridFunctionCoefficient(u_alpha_gf)) [+ MassIntegrator(1)]: the
// conductivity field is a grid function on the form's own space (ECM2_COEFF_GRIDFUNC), re-read at
// every Assemble (ConductionOperator::SetParameters, examples/ex16p.cpp:450-466)
static ecm2_pa_form *make_ex16_form(int ne, int order, int ndofs, const std::vector<int> &gmap,
                                    const std::vector<double> &enodes, bool mass, const double *ua_dev)
{
   ecm2_pa_form *f = nullptr;
   const double one = 1.0;
   CHECK(ecm2_pa_form_create(ne, order, ndofs, gmap.data(), 0, &f));
   CHECK(ecm2_pa_form_set_element_nodes(f, enodes.data()));
   if (mass) { CHECK(ecm2_pa_form_add_integrator(f, ECM2_MASS, ECM2_COEFF_CONSTANT, &one, nullptr)); }
   CHECK(ecm2_pa_form_add_integrator(f, ECM2_DIFFUSION, ECM2_COEFF_GRIDFUNC, ua_dev, nullptr));
   CHECK(ecm2_pa_form_assemble(f, nullptr));
   return f;
}

int main(int argc, char **argv)
{
   const std::string path = argc > 1 ? argv[1] : "tests/golden/fichera.mesh";
   const int refine = argc > 2 ? std::atoi(argv[2]) : 2;
   const int order = argc > 3 ? std::atoi(argv[3]) : 2;
   const int steps = argc > 4 ? std::atoi(argv[4]) : 5;

   ecm2_mesh *mesh = nullptr;
   CHECK(ecm2_mesh_read(path.c_str(), &mesh));
   for (int i = 0; i < refine; i++) { CHECK(ecm2_mesh_refine_uniform(mesh)); }
   ecm2_h1space *fes = nullptr;
   CHECK(ecm2_h1space_create(mesh, order, ECM2_NUMBERING_ENTITY, &fes));
   int ndofs = 0, ne = 0, nd = 0;
   CHECK(ecm2_h1space_info(fes, &ndofs, &ne, &nd));
   std::vector<int> gmap((size_t)ne * nd);
   CHECK(ecm2_h1space_get_gather_map(fes, gmap.data()));
   std::vector<double> enodes((size_t)ne * 24), X((size_t)ndofs * 3);
   CHECK(ecm2_mesh_get_element_nodes(mesh, enodes.data()));
   CHECK(ecm2_h1space_dof_coords(fes, mesh, X.data()));
   int n_ess = 0;
   CHECK(ecm2_h1space_boundary_dofs(fes, nullptr, &n_ess));
   std::vector<int> ess(n_ess);
   CHECK(ecm2_h1space_boundary_dofs(fes, ess.data(), &n_ess));
   std::printf("mesh %s refined %d: %d elements, H1 p=%d, %d dofs, %d boundary dofs\n", path.c_str(), refine, ne,
               order, ndofs, n_ess);

   // the first compute entry point: with no HIP device it fails here (ECM2_ERR_HIP), no fallback
   ecm2_pa_form *M1 = make_form(ne, order, ndofs, gmap, enodes, 1.0, false, nullptr, 0.0);

   // initial temperature: a hot spot at the origin over 37 C (the bench's T field)
   std::vector<double> T0(ndofs);
   for (int i = 0; i < ndofs; i++)
   {
      const double *p = &X[3 * (size_t)i];
      T0[i] = 37.0 + 20.0 * std::exp(-10.0 * (p[0] * p[0] + p[1] * p[1] + p[2] * p[2]));
   }
   double *T = device_copy(T0);
   int *ess_d = device_copy(ess);
   std::vector<double> ones(ndofs, 1.0);
   double *one = device_copy(ones);
   double *y = nullptr;
   HIPCHECK(hipMalloc(&y, ndofs * sizeof(double)));

   // known answers on the reference's fichera fixture (7 unit cubes)
   bool pass = true;
   {
      CHECK(ecm2_pa_form_mult(M1, one, y, nullptr));
      const std::vector<double> m = host_copy(y, ndofs);
      double vol = 0.0;
      for (double v : m) { vol += v; }
      ecm2_pa_form *K1 = make_form(ne, order, ndofs, gmap, enodes, 0.0, true, T, 1.0);
      CHECK(ecm2_pa_form_mult(K1, one, y, nullptr));
      const std::vector<double> k = host_copy(y, ndofs);
      double kmax = 0.0;
      for (double v : k) { kmax = std::max(kmax, std::fabs(v)); }
      std::printf("1^T M 1 = %.15f (|fichera| = 7 for the fixture), max |K 1| = %.3e\n", vol, kmax);
      if (path.find("fichera") != std::string::npos) { pass &= std::fabs(vol - 7.0) < 1e-11; }
      pass &= kmax < 1e-11;
      ecm2_pa_form_destroy(K1);
      ecm2_pa_form_destroy(M1);
   }

   // ex16p: M du/dt = -K(u) u with K(u) = div((kappa + alpha u) grad), rho c = 1 (scaled), SDIRK33
   // stages (M + c dt K) k = -K u; as ex16p, the conductivity is lagged: SetParameters(u) after
   // every step forms u_alpha_gf = kappa + alpha u at the dofs and re-assembles K and T from it
   const int type = 23;
   const double dt = 0.01, c = ecm2_ode_implicit_coeff(type), kappa = 0.5, alpha_u = 0.01;
   // u = T - 37 (the excess temperature decays to the boundary value 0)
   std::vector<double> u0(ndofs);
   for (int i = 0; i < ndofs; i++) { u0[i] = T0[i] - 37.0; }
   for (int i : ess) { u0[i] = 0.0; }
   double *u = device_copy(u0);
   std::vector<double> ua(ndofs), cua(ndofs);
   auto set_parameters = [&](const std::vector<double> &uh) {
      for (int i = 0; i < ndofs; i++)
      {
         ua[i] = kappa + alpha_u * uh[i];
         cua[i] = c * dt * ua[i];
      }
   };
   set_parameters(u0);
   double *ua_d = device_copy(ua), *cua_d = device_copy(cua);
   ecm2_pa_form *Kf = make_ex16_form(ne, order, ndofs, gmap, enodes, false, ua_d);
   ecm2_pa_form *Tf = make_ex16_form(ne, order, ndofs, gmap, enodes, true, cua_d);
   int snap = 0, mvals = 0, atpt = 0;
   CHECK(ecm2_pa_form_snapshot_info(Tf, &snap, &mvals, &atpt));
   std::printf("T = M + c dt K(u): coefficient snapshot %d (mass values %d, laws at the point %d)\n", snap, mvals,
               atpt);
   ecm2_operator *Kop = nullptr, *Top = nullptr;
   CHECK(ecm2_operator_from_pa_form(Kf, &Kop));
   CHECK(ecm2_operator_from_pa_form(Tf, &Top));
   double umax0 = 0.0;
   for (double v : u0) { umax0 = std::max(umax0, std::fabs(v)); }
   double umax = umax0;
   for (int s = 0; s < steps; s++)
   {
      int solves = 0, iters = 0, conv = 0;
      CHECK(ecm2_ode_step(type, Top, Kop, dt, u, ess_d, n_ess, 1e-12, 2000, 1, &solves, &iters, &conv, nullptr));
      const std::vector<double> uh = host_copy(u, ndofs);
      double mx = 0.0;
      for (double v : uh) { mx = std::max(mx, std::fabs(v)); }
      std::printf("step %d: %d stage solves, %d PCG iterations, converged %d, max |u| = %.6f\n", s + 1, solves,
                  iters, conv, mx);
      pass &= conv != 0 && std::isfinite(mx) && mx <= umax * (1.0 + 1e-12);  // a heat equation's maximum principle
      umax = mx;
      // ConductionOperator::SetParameters(u): the new conductivity field, then Assemble (the forms
      // read their grid functions at Assemble, as the reference's K->Assemble does)
      set_parameters(uh);
      HIPCHECK(hipMemcpy(ua_d, ua.data(), ndofs * sizeof(double), hipMemcpyHostToDevice));
      HIPCHECK(hipMemcpy(cua_d, cua.data(), ndofs * sizeof(double), hipMemcpyHostToDevice));
      CHECK(ecm2_pa_form_assemble(Kf, nullptr));
      CHECK(ecm2_pa_form_assemble(Tf, nullptr));
   }
   pass &= umax < umax0;
   std::printf("%s\n", pass ? "PASS" : "FAIL");

   ecm2_operator_destroy(Top);
   ecm2_operator_destroy(Kop);
   ecm2_pa_form_destroy(Tf);
   ecm2_pa_form_destroy(Kf);
   (void)hipFree(u);
   (void)hipFree(ua_d);
   (void)hipFree(cua_d);
   (void)hipFree(y);
   (void)hipFree(one);
   (void)hipFree(ess_d);
   (void)hipFree(T);
   ecm2_h1space_destroy(fes);
   ecm2_mesh_destroy(mesh);
   return pass ? 0 : 1;
}
