// par_heat.cpp -- the parallel side of examples/ex16p.cpp (ParBilinearForm at
// AssemblyLevel::PARTIAL over a z-slab partition, the RAPOperator Mult and an SDIRK step on
// it) through the C ABI alone: N subdomains of a Cartesian mesh as an in-process loopback group
// on one GPU (ecm2_par_group_*, the exchange as device copies that follow the same exchange
// schedule the RCCL transport sends).  `par_heat rccl ...` is the one-process-per-GPU form: each
// process (RANK, WORLD_SIZE, LOCAL_RANK from the environment, as torchrun sets them) builds its
// own rank's partition and form with an RCCL id (ecm2_rccl_unique_id on rank 0, handed to the
// others through the file ECM2_ID_FILE names) and uses ecm2_par_form_mult /
// ecm2_operator_from_par_form; PCG dots are summed over the ranks with ncclAllReduce.
// Checks, against the serial form on the whole mesh: the Mult on the true dofs (rank by rank)
// and two SDIRK33 steps.  Exit status 0 = pass.
//
// Usage: par_heat [subdomains = 4] [n = 12 elements per edge] [order = 2] [decomposition = 1 (OVERLAP), 0 RAP]
//        RANK=r WORLD_SIZE=N ECM2_ID_FILE=path par_heat rccl [n] [order] [decomposition]
#include "ecm2_pa.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <chrono>
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

static std::vector<double> host_copy(const double *d, size_t n)
{
   std::vector<double> h(n);
   HIPCHECK(hipMemcpy(h.data(), d, n * sizeof(double), hipMemcpyDeviceToHost));
   return h;
}

static const double kSlope = 0.0012, kTref = 37.0;

struct Rank
{
   ecm2_partition *part = nullptr;
   int ne_local = 0, n_owned = 0, n_ghost = 0, offset = 0;
   std::vector<int> elems, l2g;
   std::vector<double> enodes;
   double *T = nullptr;  // local L-vector of the temperature [owned | ghost]
};

static int env_int(const char *name, int dflt)
{
   const char *v = std::getenv(name);
   return v ? std::atoi(v) : dflt;
}

// one RCCL id per communicator (each par form holds its own): rank 0 makes kForms ids and
// publishes them with the job's nonce (write + rename); the others wait for a file carrying
// their own nonce, so a file left over from an earlier job is never read as this job's ids.
// The nonce is ECM2_JOB_ID, else the launcher's TORCHELASTIC_RUN_ID, else MASTER_ADDR:PORT.
constexpr int kForms = 3, kNonce = 128;
static std::string job_nonce()
{
   for (const char *k : {"ECM2_JOB_ID", "TORCHELASTIC_RUN_ID"})
   {
      const char *v = std::getenv(k);
      if (v && *v) { return v; }
   }
   const char *a = std::getenv("MASTER_ADDR"), *p = std::getenv("MASTER_PORT");
   return (a && p) ? std::string(a) + ":" + p : std::string();
}

static bool share_rccl_id(int rank, int world, unsigned char *id)
{
   if (rank == 0)
   {
      for (int k = 0; k < kForms; k++) { CHECK(ecm2_rccl_unique_id(id + 128 * k)); }
   }
   if (world == 1) { return true; }
   const char *path = std::getenv("ECM2_ID_FILE");
   const std::string nonce = job_nonce();
   if (!path || nonce.empty() || nonce.size() >= (size_t)kNonce)
   {
      std::fprintf(stderr, "WORLD_SIZE > 1 needs ECM2_ID_FILE (a path all ranks can read) and a job nonce "
                           "(ECM2_JOB_ID, TORCHELASTIC_RUN_ID or MASTER_ADDR/MASTER_PORT)\n");
      return false;
   }
   char tag[kNonce] = {};
   std::memcpy(tag, nonce.data(), nonce.size());
   if (rank == 0)
   {
      const std::string tmp = std::string(path) + ".tmp";
      FILE *f = std::fopen(tmp.c_str(), "wb");
      if (!f || std::fwrite(tag, 1, kNonce, f) != kNonce || std::fwrite(id, 1, 128 * kForms, f) != 128 * kForms ||
          std::fclose(f) != 0)
      {
         return false;
      }
      return std::rename(tmp.c_str(), path) == 0;
   }
   for (int t = 0; t < 12000; t++)  // 120 s
   {
      if (FILE *f = std::fopen(path, "rb"))
      {
         char got_tag[kNonce];
         const size_t gt = std::fread(got_tag, 1, kNonce, f);
         const size_t got = gt == kNonce ? std::fread(id, 1, 128 * kForms, f) : 0;
         std::fclose(f);
         if (got == 128 * kForms && std::memcmp(got_tag, tag, kNonce) == 0) { return true; }  // else: stale
      }
      std::this_thread::sleep_for(std::chrono::milliseconds(10));
   }
   return false;
}

int main(int argc, char **argv)
{
   const bool rccl = argc > 1 && std::strcmp(argv[1], "rccl") == 0;
   // argv[1] is the subdomain count or "rccl"; then n, order, decomposition in both forms
   const int my_rank = rccl ? env_int("RANK", 0) : -1;
   const int N = rccl ? env_int("WORLD_SIZE", 1) : (argc > 1 ? std::atoi(argv[1]) : 4);
   const int n = argc > 2 ? std::atoi(argv[2]) : 12;
   const int order = argc > 3 ? std::atoi(argv[3]) : 2;
   const int decomp = argc > 4 ? std::atoi(argv[4]) : ECM2_DECOMP_OVERLAP;

   if (ecm2_device_count() <= 0)
   {
      std::fprintf(stderr, "no HIP device available (the PA path has no CPU fallback)\n");
      return 2;
   }
   unsigned char id[128 * kForms] = {};
   if (rccl)
   {
      HIPCHECK(hipSetDevice(env_int("LOCAL_RANK", my_rank) % ecm2_device_count()));
      if (!share_rccl_id(my_rank, N, id))
      {
         std::fprintf(stderr, "rank %d: no RCCL id\n", my_rank);
         return 2;
      }
   }
   ecm2_mesh *mesh = nullptr;
   CHECK(ecm2_mesh_cartesian(n, n, n, 1.0, 1.0, 1.0, &mesh));
   ecm2_h1space *fes = nullptr;
   CHECK(ecm2_h1space_create(mesh, order, ECM2_NUMBERING_STRUCTURED, &fes));
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
   std::vector<char> is_ess(ndofs, 0);
   for (int d : ess) { is_ess[d] = 1; }

   // global fields: temperature (a hot spot over 37 C) and a test vector
   std::vector<double> Tg(ndofs), xg(ndofs);
   for (int i = 0; i < ndofs; i++)
   {
      const double *p = &X[3 * (size_t)i];
      const double r2 = (p[0] - 0.5) * (p[0] - 0.5) + (p[1] - 0.5) * (p[1] - 0.5) + (p[2] - 0.5) * (p[2] - 0.5);
      Tg[i] = kTref + 20.0 * std::exp(-20.0 * r2);
      xg[i] = std::sin(3.0 * p[0] + 1.0) * std::cos(2.0 * p[1]) + p[2];
   }
   double *T = device_copy(Tg);

   // serial reference forms on the whole mesh: A = M + K(T), K(T), and T_ode = M + c dt K(T)
   const int type = 23;
   const double dt = 0.002, c = ecm2_ode_implicit_coeff(type);
   auto serial_form = [&](double alpha, double kscale) {
      ecm2_pa_form *f = nullptr;
      CHECK(ecm2_pa_form_create(ne, order, ndofs, gmap.data(), 0, &f));
      CHECK(ecm2_pa_form_set_element_nodes(f, enodes.data()));
      if (alpha != 0.0) { CHECK(ecm2_pa_form_add_integrator(f, ECM2_MASS, ECM2_COEFF_CONSTANT, &alpha, nullptr)); }
      const double params[3] = {kscale, kSlope, kTref};
      CHECK(ecm2_pa_form_add_integrator(f, ECM2_DIFFUSION, ECM2_COEFF_GRIDFUNC_AFFINE, T, params));
      CHECK(ecm2_pa_form_assemble(f, nullptr));
      return f;
   };

   // the partition: z-slabs (Mesh::CartesianPartitioning along z), one local space per rank
   std::vector<int> elem_rank(ne);
   CHECK(ecm2_partition_slabs_z(mesh, N, elem_rank.data()));
   // the group builds every rank's local space; an RCCL process only its own
   std::vector<Rank> ranks(rccl ? 1 : N);
   int n_true = 0;
   for (int k = 0; k < (int)ranks.size(); k++)
   {
      const int r = rccl ? my_rank : k;
      Rank &R = ranks[k];
      CHECK(ecm2_partition_create_ex(fes, mesh, elem_rank.data(), r, N, decomp, &R.part));
      int ne_int = 0, n_nbrs = 0, n_send = 0;
      CHECK(ecm2_partition_info(R.part, &R.ne_local, &ne_int, &R.n_owned, &R.n_ghost, &n_nbrs, &n_send));
      R.elems.resize(R.ne_local);
      R.l2g.resize((size_t)R.n_owned + R.n_ghost);
      CHECK(ecm2_partition_get(R.part, R.elems.data(), R.l2g.data(), nullptr, nullptr, nullptr, nullptr, nullptr));
      R.enodes.resize((size_t)R.ne_local * 24);
      for (int e = 0; e < R.ne_local; e++)
      {
         std::copy_n(&enodes[(size_t)R.elems[e] * 24], 24, &R.enodes[(size_t)e * 24]);
      }
      std::vector<double> Tl(R.l2g.size());
      for (size_t i = 0; i < Tl.size(); i++) { Tl[i] = Tg[R.l2g[i]]; }
      R.T = device_copy(Tl);
      R.offset = n_true;
      n_true += R.n_owned;
      std::printf("rank %d: %d local elements (%d interior), %d owned + %d ghost dofs, %d neighbours\n", r,
                  R.ne_local, ne_int, R.n_owned, R.n_ghost, n_nbrs);
   }
   if (!rccl && n_true != ndofs)
   {
      std::fprintf(stderr, "owned dofs %d != %d\n", n_true, ndofs);
      return 1;
   }
   const int NL = (int)ranks.size();
   int next_id = 0;  // RCCL: the next unused communicator id
   auto par_forms = [&](double alpha, double kscale) {
      unsigned char *fid = rccl ? id + 128 * next_id++ : nullptr;
      if (next_id > kForms) { std::fprintf(stderr, "out of RCCL ids\n"); std::exit(2); }
      std::vector<ecm2_par_form *> fs(NL);
      for (int r = 0; r < NL; r++)
      {
         CHECK(ecm2_par_form_create(ranks[r].part, ranks[r].enodes.data(), 0, fid, &fs[r]));
         if (alpha != 0.0)
         {
            CHECK(ecm2_par_form_add_integrator(fs[r], ECM2_MASS, ECM2_COEFF_CONSTANT, &alpha, nullptr));
         }
         const double params[3] = {kscale, kSlope, kTref};
         CHECK(ecm2_par_form_add_integrator(fs[r], ECM2_DIFFUSION, ECM2_COEFF_GRIDFUNC_AFFINE, ranks[r].T, params));
         CHECK(ecm2_par_form_assemble(fs[r], nullptr));
      }
      return fs;
   };
   // concatenated true vector (rank r's owned dofs at its offset) <-> global dofs
   auto to_true = [&](const std::vector<double> &g) {
      std::vector<double> t(n_true);
      for (const Rank &R : ranks)
         for (int i = 0; i < R.n_owned; i++) { t[R.offset + i] = g[R.l2g[i]]; }
      return t;
   };
   auto rel_diff = [&](const std::vector<double> &t, const std::vector<double> &g) {
      double num = 0.0, den = 0.0;
      for (const Rank &R : ranks)
         for (int i = 0; i < R.n_owned; i++)
         {
            num = std::max(num, std::fabs(t[R.offset + i] - g[R.l2g[i]]));
            den = std::max(den, std::fabs(g[R.l2g[i]]));
         }
      return num / std::max(den, 1e-300);
   };
   bool pass = true;

   // (1) the operator: group Mult == serial Mult, rank by rank
   {
      ecm2_pa_form *A = serial_form(1.0, 1.0);
      double *x = device_copy(xg), *y = nullptr;
      HIPCHECK(hipMalloc(&y, ndofs * sizeof(double)));
      CHECK(ecm2_pa_form_mult(A, x, y, nullptr));
      const std::vector<double> ys = host_copy(y, ndofs);
      std::vector<ecm2_par_form *> fs = par_forms(1.0, 1.0);
      const std::vector<double> xt = to_true(xg);
      std::vector<const double *> xr(NL);
      std::vector<double *> yr(NL);
      double *xtd = device_copy(xt), *ytd = nullptr;
      HIPCHECK(hipMalloc(&ytd, std::max(1, n_true) * sizeof(double)));
      for (int r = 0; r < NL; r++) { xr[r] = xtd + ranks[r].offset; yr[r] = ytd + ranks[r].offset; }
      if (rccl) { CHECK(ecm2_par_form_mult(fs[0], xtd, ytd, nullptr)); }  // collective over the ranks
      else { CHECK(ecm2_par_group_mult(fs.data(), N, xr.data(), yr.data(), nullptr)); }
      const double e = rel_diff(host_copy(ytd, n_true), ys);
      std::printf("%s Mult vs serial: max rel diff %.3e (%s decomposition, %d subdomains)\n",
                  rccl ? "RCCL rank" : "group", e, decomp == ECM2_DECOMP_OVERLAP ? "OVERLAP" : "RAP", N);
      pass &= e < 1e-12;
      for (ecm2_par_form *f : fs) { ecm2_par_form_destroy(f); }
      (void)hipFree(ytd);
      (void)hipFree(xtd);
      (void)hipFree(y);
      (void)hipFree(x);
      ecm2_pa_form_destroy(A);
   }

   // (2) ex16p's time step: SDIRK33 on the group operators == on the serial operators
   {
      std::vector<double> u0(ndofs);
      for (int i = 0; i < ndofs; i++) { u0[i] = is_ess[i] ? 0.0 : Tg[i] - kTref; }
      ecm2_pa_form *Ks = serial_form(0.0, 0.5), *Ts = serial_form(1.0, c * dt * 0.5);
      ecm2_operator *Kop = nullptr, *Top = nullptr;
      CHECK(ecm2_operator_from_pa_form(Ks, &Kop));
      CHECK(ecm2_operator_from_pa_form(Ts, &Top));
      double *us = device_copy(u0);
      int *ess_d = device_copy(ess);
      std::vector<ecm2_par_form *> Kp = par_forms(0.0, 0.5), Tp = par_forms(1.0, c * dt * 0.5);
      ecm2_operator *Kg = nullptr, *Tgop = nullptr;
      if (rccl)
      {
         CHECK(ecm2_operator_from_par_form(Kp[0], &Kg));
         CHECK(ecm2_operator_from_par_form(Tp[0], &Tgop));
      }
      else
      {
         CHECK(ecm2_operator_from_par_group(Kp.data(), N, &Kg));
         CHECK(ecm2_operator_from_par_group(Tp.data(), N, &Tgop));
      }
      int gsize = 0;
      CHECK(ecm2_operator_size(Kg, &gsize));
      pass &= gsize == n_true;
      std::vector<int> ess_t;
      for (const Rank &R : ranks)
         for (int i = 0; i < R.n_owned; i++) { if (is_ess[R.l2g[i]]) { ess_t.push_back(R.offset + i); } }
      int *ess_td = device_copy(ess_t);
      double *ut = device_copy(to_true(u0));
      for (int s = 0; s < 2; s++)
      {
         int solves = 0, its = 0, conv = 0, gsolves = 0, gits = 0, gconv = 0;
         CHECK(ecm2_ode_step(type, Top, Kop, dt, us, ess_d, n_ess, 1e-12, 2000, 1, &solves, &its, &conv, nullptr));
         CHECK(ecm2_ode_step(type, Tgop, Kg, dt, ut, ess_td, (int)ess_t.size(), 1e-12, 2000, 1, &gsolves, &gits,
                             &gconv, nullptr));
         const double e = rel_diff(host_copy(ut, n_true), host_copy(us, ndofs));
         std::printf("step %d: serial %d PCG iterations, group %d; max rel diff %.3e\n", s + 1, its, gits, e);
         pass &= conv && gconv && e < 1e-9;
      }
      (void)hipFree(ut);
      (void)hipFree(ess_td);
      ecm2_operator_destroy(Tgop);
      ecm2_operator_destroy(Kg);
      for (ecm2_par_form *f : Tp) { ecm2_par_form_destroy(f); }
      for (ecm2_par_form *f : Kp) { ecm2_par_form_destroy(f); }
      (void)hipFree(ess_d);
      (void)hipFree(us);
      ecm2_operator_destroy(Top);
      ecm2_operator_destroy(Kop);
      ecm2_pa_form_destroy(Ts);
      ecm2_pa_form_destroy(Ks);
   }
   if (rccl) { std::printf("rank %d of %d: ", my_rank, N); }
   std::printf("%s\n", pass ? "PASS" : "FAIL");

   for (Rank &R : ranks)
   {
      (void)hipFree(R.T);
      ecm2_partition_destroy(R.part);
   }
   (void)hipFree(T);
   ecm2_h1space_destroy(fes);
   ecm2_mesh_destroy(mesh);
   return pass ? 0 : 1;
}
