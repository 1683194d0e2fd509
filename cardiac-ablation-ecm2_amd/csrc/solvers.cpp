// solvers.cpp -- see solvers.hpp.
#include "solvers.hpp"

#include <thread>

#include <algorithm>
#include <cmath>
#include <memory>

namespace ecm2
{

// ---------------------------------------------------------------------------------------
// loopback group as one operator
// ---------------------------------------------------------------------------------------
GroupOp::GroupOp(std::vector<ParPAForm *> forms) : forms_(std::move(forms))
{
   off_.assign(forms_.size() + 1, 0);
   for (size_t r = 0; r < forms_.size(); r++) { off_[r + 1] = off_[r] + forms_[r]->true_size(); }
   n_ = off_.back();
}

void GroupOp::mult(const double *x, double *y, hipStream_t s)
{
   std::vector<const double *> xs;
   std::vector<double *> ys;
   for (size_t r = 0; r < forms_.size(); r++)
   {
      xs.push_back(x + off_[r]);
      ys.push_back(y + off_[r]);
   }
   par_group_mult(forms_, xs, ys, s);
}

void GroupOp::diagonal(double *d, hipStream_t s)
{
   std::vector<double *> ds;
   for (size_t r = 0; r < forms_.size(); r++) { ds.push_back(d + off_[r]); }
   par_group_diagonal(forms_, ds, s);
}

MemberOp::MemberOp(std::vector<ParPAForm *> forms, int member) : forms_(std::move(forms)), member_(member)
{
   const int n = (int)forms_.size();
   ECM2_VERIFY(member >= 0 && member < n, ERR_ARG, "member " << member << " outside the group of " << n);
   // the peers' x live in this operator's own buffer, on which no group Mult runs: their packed sends
   // and (RAP) their ghost sums would be stale
   ECM2_VERIFY(forms_[member]->part().overlap, ERR_UNSUPPORTED, "a member operator needs the OVERLAP decomposition");
   for (ParPAForm *f : forms_)
   {
      ECM2_VERIFY(!f->pack_needed(), ERR_UNSUPPORTED, "a member operator needs contiguous sends (slabs)");
   }
   off_.assign(n + 1, 0);
   for (int r = 0; r < n; r++) { off_[r + 1] = off_[r] + forms_[r]->true_size(); }
   peers_.resize(std::max(off_.back(), 1));
   yscratch_.resize(std::max(off_.back(), 1));
   ECM2_HIP(hipMemset(peers_.data(), 0, peers_.size() * sizeof(double)));
}

void MemberOp::mult(const double *x, double *y, hipStream_t s)
{
   std::vector<const double *> xs;
   std::vector<double *> ys;
   for (size_t r = 0; r < forms_.size(); r++)
   {
      const bool me = (int)r == member_;
      xs.push_back(me ? x : peers_.data() + off_[r]);
      ys.push_back(me ? y : yscratch_.data() + off_[r]);
   }
   par_group_mult_member(forms_, xs, ys, member_, s);
}

void MemberOp::diagonal(double *d, hipStream_t s)
{
   std::vector<double *> ds;
   for (size_t r = 0; r < forms_.size(); r++) { ds.push_back(yscratch_.data() + off_[r]); }
   par_group_diagonal(forms_, ds, s);
   const int n = size();
   if (n) { ECM2_HIP(hipMemcpyAsync(d, ds[member_], n * sizeof(double), hipMemcpyDeviceToDevice, s)); }
}

// ---------------------------------------------------------------------------------------
// ConstrainedOperator + CGSolver + OperatorJacobiSmoother
// ---------------------------------------------------------------------------------------
namespace
{
// CGSolver's work vectors live across solves (CGSolver::SetOperator allocates them once,
// solvers.cpp:869-880): one workspace per host thread and device, grown on demand, with a
// mapped pinned scalar the final-dot kernels write the stopping-test value into.
struct PCGWork
{
   DeviceArray<double> r, d, z, saved, dinv, partials, scal;
   double *hs = nullptr, *hs_dev = nullptr;
   DeviceArray<kern::PcgCtl> ctl;                          // the device-driven loop's state
   kern::PcgCtl *hctl = nullptr, *hctl_dev = nullptr;      // its mapped pinned mirror
   ~PCGWork()
   {
      if (hs) { (void)hipHostFree(hs); }
      if (hctl) { (void)hipHostFree(hctl); }
   }
   void ensure(int n, int n_ess, bool jacobi)
   {
      auto grow = [](DeviceArray<double> &a, size_t m) {
         if (a.size() < m) { a.resize(m); }
      };
      grow(r, std::max(n, 1));
      grow(d, std::max(n, 1));
      grow(z, std::max(n, 1));
      grow(saved, std::max(n_ess, 1));
      if (jacobi) { grow(dinv, std::max(n, 1)); }
      grow(partials, kern::kDotPartials);
      grow(scal, 4);
      if (!hs)
      {
         ECM2_HIP(hipHostMalloc(&hs, 4 * sizeof(double), hipHostMallocMapped));
         ECM2_HIP(hipHostGetDevicePointer(reinterpret_cast<void **>(&hs_dev), hs, 0));
         // (coherent: the host polls it while kernels run)
         ECM2_HIP(hipHostMalloc(&hctl, sizeof(kern::PcgCtl), hipHostMallocMapped | hipHostMallocCoherent));
         ECM2_HIP(hipHostGetDevicePointer(reinterpret_cast<void **>(&hctl_dev), hctl, 0));
         ctl.resize(1);
      }
   }
};

PCGWork &pcg_work()
{
   static thread_local std::vector<std::unique_ptr<PCGWork>> per_device;
   int dev = 0;
   ECM2_HIP(hipGetDevice(&dev));
   if ((int)per_device.size() <= dev) { per_device.resize(dev + 1); }
   if (!per_device[dev]) { per_device[dev].reset(new PCGWork()); }
   return *per_device[dev];
}
} // namespace

PCGResult pcg_solve(LinOp &A, const int *ess, int n_ess, const double *b, double *x, double rel_tol,
                    double abs_tol, int max_iter, bool jacobi, hipStream_t s)
{
   const int n = A.size();
   PCGResult res;
   PCGWork &w = pcg_work();
   w.ensure(n, n_ess, jacobi);
   double *r = w.r.data(), *d = w.d.data(), *z = w.z.data(), *dinv = jacobi ? w.dinv.data() : nullptr;
   double *partials = w.partials.data();
   // device scalars; nom and betanom swap roles every iteration (no copy); alpha of the last step
   double *nom = w.scal.data(), *den = w.scal.data() + 1, *betanom = w.scal.data() + 2, *alpha = w.scal.data() + 3;
   // serial: the final-dot kernel also writes the value into mapped pinned memory, so the
   // stopping test needs only a stream sync; distributed: copy after the all-reduce
   const bool direct = !A.distributed();
   auto dot = [&](const double *a, const double *bb, double *out, const kern::PcgCtl *c = nullptr) {
      kern::dot(n, a, bb, partials, out, s, direct && !c ? w.hs_dev : nullptr, c);
      A.sum_scalars(out, 1, s);
   };
   auto readback = [&](const double *dv) {
      if (!direct) { ECM2_HIP(hipMemcpyAsync(w.hs, dv, sizeof(double), hipMemcpyDeviceToHost, s)); }
      ECM2_HIP(hipStreamSynchronize(s));
      return *(volatile double *)w.hs;
   };
   // ConstrainedOperator::ConstrainedMult, DIAG_ONE (operator.cpp:586-646): the input's
   // ess entries are zeroed in place for the Mult and restored after (no vector copy);
   // out[ess] = in[ess]
   auto cmult = [&](double *in, double *out) {
      if (n_ess == 0) { A.mult(in, out, s); return; }
      kern::ess_save_zero(n_ess, ess, in, w.saved.data(), s);
      A.mult(in, out, s);
      kern::ess_restore(n_ess, ess, w.saved.data(), in, out, s);
   };
   // den = (A d, d) folded into the Mult where the operator can (serial snapshot forms): the
   // kernel's element energies sum_e d~_e . A_e d~_e (d~ = d with the ess entries zeroed, as the
   // constrained Mult sees it) plus the DIAG_ONE rows' sum_ess d_i^2 -- the same value as the dot of
   // d and A d up to the summation order -- one partial per workgroup, summed in a fixed order by
   // dot_final: no pass over the two vectors (2 streams and a launch per iteration).
   const int nen = direct ? A.energy_parts() : 0;
   const int nparts = std::max({kern::kDotPartials, kern::step_parts(n), nen + kern::ess_parts(n_ess)});
   if ((int)w.partials.size() < nparts)
   {
      w.partials.resize(nparts);
      partials = w.partials.data();
   }
   auto cmult_den = [&](double *in, double *out, const kern::PcgCtl *c, const kern::PcgStop *stop) {
      if (n_ess) { kern::ess_save_zero(n_ess, ess, in, w.saved.data(), s); }
      A.mult_energy(in, out, partials, s);
      if (n_ess) { kern::ess_restore(n_ess, ess, w.saved.data(), in, out, s, partials + nen); }
      kern::dot_final(nen + kern::ess_parts(n_ess), partials, den, s, c, stop, c ? nullptr : w.hs_dev);
   };
   if (jacobi)
   {
      // OperatorJacobiSmoother on the constrained operator: ess rows get diag 1
      A.diagonal(z, s);
      if (n_ess) { kern::set_values(n_ess, ess, 1.0, z, s); }
      kern::reciprocal(n, z, dinv, s);
   }
   if (n) { ECM2_HIP(hipMemcpyAsync(r, b, sizeof(double) * n, hipMemcpyDeviceToDevice, s)); }
   if (n) { ECM2_HIP(hipMemsetAsync(x, 0, sizeof(double) * n, s)); }
   if (jacobi)
   {
      kern::pcg_precond(n, dinv, r, z, s);
      if (n) { ECM2_HIP(hipMemcpyAsync(d, z, sizeof(double) * n, hipMemcpyDeviceToDevice, s)); }
   }
   else if (n)
   {
      ECM2_HIP(hipMemcpyAsync(d, r, sizeof(double) * n, hipMemcpyDeviceToDevice, s));
   }
   dot(d, r, nom);
   const double nom0 = readback(nom);
   // CGSolver::Mult's checks before the loop (solvers.cpp:893-948)
   ECM2_VERIFY(std::isfinite(nom0), ERR_NUMERIC, "PCG: nom = " << nom0);
   res.initial_norm = nom0 >= 0 ? std::sqrt(nom0) : nom0;
   res.final_norm = res.initial_norm;
   if (nom0 < 0.0)
   {
      // the preconditioner is not positive definite: not converged, final_norm = nom (:905-917)
      res.initial_norm = res.final_norm = nom0;
      ECM2_HIP(hipStreamSynchronize(s));
      return res;
   }
   const double r0 = std::max(nom0 * rel_tol * rel_tol, abs_tol * abs_tol);
   if (nom0 <= r0) { res.converged = true; }
   else
   {
      // the device-driven loop's state, reset before the read-back below idles the stream (no
      // kernel of a previous solve writes the mirror any more: every solve ends synchronised)
      ECM2_HIP(hipMemsetAsync(w.ctl.data(), 0, sizeof(kern::PcgCtl), s));
      *w.hctl = kern::PcgCtl{};
      if (nen > 0) { cmult_den(d, z, nullptr, nullptr); }
      else
      {
         cmult(d, z);
         dot(z, d, den);
      }
      const double den0 = readback(den);
      ECM2_VERIFY(std::isfinite(den0), ERR_NUMERIC, "PCG: den = " << den0);
      if (den0 != 0.0)
      {
         // CGSolver's loop (solvers.cpp:930-1000) driven by the device: the stopping tests run on
         // the device after each r.z and each (A d, d) (in the dot's final pass, or in a one-thread
         // kernel after the all-reduce), and once one stops every later vector kernel returns at once.
         // The host enqueues iteration i as soon as the betanom test of i - 1 has run (it polls the
         // mirror's progress mark; no host synchronisation of the stream), so the queue holds the
         // rest of iteration i - 1 while it does, and it ends at the iteration the device stopped at:
         // the same iteration on every rank, so the ranks issue the same collectives.  The iterates
         // are CGSolver's (the same operations per entry, in its order; x += alpha d deferred into
         // the next pass that reads d); at most the stopping iteration's Mult runs after the stop.
         kern::PcgCtl *ctl = w.ctl.data(), *hm = w.hctl;
         auto vol = [](const int &v) { return *(volatile const int *)&v; };
         // has the loop stopped at an iteration <= waited?  (waits until the test of `waited` ran)
         auto stopped_by = [&](int waited) {
            for (long spin = 1;; spin++)
            {
               if (vol(hm->checked) >= waited)
               {
                  // (the device writes done before checked: a stop at `waited` is visible now)
                  return vol(hm->done) != 0 && vol(hm->iters) <= waited;
               }
               if (vol(hm->done) != 0) { return vol(hm->iters) <= waited; }
               if (spin % 4096 == 0)
               {
                  const hipError_t e = hipStreamQuery(s);
                  if (e == hipSuccess && vol(hm->checked) < waited && vol(hm->done) == 0)
                  {
                     ECM2_VERIFY(false, ERR_INTERNAL, "device PCG loop: stream idle before the test of iteration " << waited);
                  }
                  if (e != hipSuccess && e != hipErrorNotReady) { ECM2_HIP(e); }
               }
               // back off after a short spin: the host core stays free for RCCL's
               // proxy and the other ranks' host threads while the device runs the iteration
               if (spin > 256) { std::this_thread::yield(); }
            }
         };
         for (int i = 1;; i++)
         {
            if (i > 1 && stopped_by(i - 1)) { break; }
            // r -= alpha A d, betanom = r.(M^{-1} r) in one pass, its test
            const kern::PcgStop stop{r0, i, max_iter, ctl, w.hctl_dev};
            kern::pcg_step_r(n, nom, den, z, r, dinv, partials, betanom, alpha, s, ctl, direct ? &stop : nullptr);
            if (!direct)
            {
               A.sum_scalars(betanom, 1, s);
               kern::pcg_check(betanom, stop, s);
            }
            if (i >= max_iter) { break; }
            // x += alpha d, d = M^{-1} r + beta d
            kern::pcg_update_xd(n, nom, den, betanom, x, d, r, dinv, s, ctl);
            // z = A d, den = (A d, d) and its test (after ++i: final_iter = i + 1 on a den == 0 stop)
            const kern::PcgStop dstop{r0, i + 1, max_iter, ctl, w.hctl_dev, betanom, 1};
            if (nen > 0) { cmult_den(d, z, ctl, &dstop); }
            else if (direct)
            {
               cmult(d, z);
               kern::dot(n, d, z, partials, den, s, nullptr, ctl, &dstop);
            }
            else
            {
               cmult(d, z);
               dot(d, z, den, ctl);
               kern::pcg_check(den, dstop, s);
            }
            std::swap(nom, betanom);  // nom <- betanom
         }
         // the stopping iteration's x += alpha d (a betanom stop)
         kern::pcg_finish_x(n, alpha, d, x, s, ctl);
         ECM2_HIP(hipStreamSynchronize(s));
         const int done = *(volatile int *)&hm->done;
         ECM2_VERIFY(done != kern::PCG_RUNNING, ERR_INTERNAL, "device PCG loop ended without a stop");
         const double bn = hm->final;
         ECM2_VERIFY(done != kern::PCG_NONFINITE, ERR_NUMERIC,
                     "PCG: non-finite (B r, r) or (A d, d) at iteration " << hm->iters << " (" << bn << ")");
         res.final_norm = bn >= 0 ? std::sqrt(bn) : bn;
         res.iterations = hm->iters;
         res.converged = done == kern::PCG_CONVERGED;
      }
   }
   ECM2_HIP(hipStreamSynchronize(s));
   return res;
}

PCGResult pcg_solve(PAForm &A, const int *ess, int n_ess, const double *b, double *x, double rel_tol,
                    double abs_tol, int max_iter, bool jacobi, hipStream_t s)
{
   FormOp op(A);
   return pcg_solve(op, ess, n_ess, b, x, rel_tol, abs_tol, max_iter, jacobi, s);
}

// ---------------------------------------------------------------------------------------
// SDIRK family (slope form, ImplicitVarType::SLOPE) on an ex16-style conduction operator
// ---------------------------------------------------------------------------------------
namespace
{
const double kSdirk33A = 0.435866521508458999416019;  // ode.cpp SDIRK33Solver::Step
const double kSdirk33B = 1.20849664917601007033648;
const double kSdirk33C = 0.717933260754229499708010;
double sdirk34_a() { return 1. / std::sqrt(3.) * std::cos(M_PI / 18.) + 0.5; }
double sdirk23_gamma(int type)
{
   return type == 22 ? (2. - std::sqrt(2.)) / 2.   // gamma_opt = 2: L-stable, order 2
                     : (3. + std::sqrt(3.)) / 6.;  // default gamma_opt: A-stable, order 3
}
} // namespace

bool ode_implicit_supported(int type)
{
   return type == 21 || type == 22 || type == 23 || type == 32 || type == 33 || type == 34;
}

double ode_implicit_coeff(int type)
{
   switch (type)
   {
      case 21: return 1.0;
      case 22:
      case 33: return sdirk23_gamma(type);
      case 23: return kSdirk33A;
      case 32: return 0.5;
      case 34: return sdirk34_a();
      default: break;
   }
   ECM2_VERIFY(false, ERR_ARG, "unsupported implicit ODE solver type " << type);
   return 0.0;
}

StepStats ode_step(int type, LinOp &T, LinOp &K, double dt, double *u, const int *ess, int n_ess,
                   double rel_tol, int max_iter, bool jacobi, hipStream_t s)
{
   ECM2_VERIFY(ode_implicit_supported(type), ERR_ARG, "unsupported implicit ODE solver type " << type);
   ECM2_VERIFY(T.size() == K.size(), ERR_ARG, "T and K sizes differ");
   const int n = T.size();
   StepStats st;
   DeviceArray<double> k(std::max(n, 1)), y(std::max(n, 1)), z(std::max(n, 1)), rhs(std::max(n, 1));
   // ConductionOperator::ImplicitSolve (ex16.cpp:327-354), slope form: T k = -K u_stage
   auto implicit_solve = [&](const double *us, double *kk) {
      K.mult(us, rhs.data(), s);
      kern::scale(n, -1.0, rhs.data(), s);
      if (n_ess) { kern::set_values(n_ess, ess, 0.0, rhs.data(), s); }
      const PCGResult r = pcg_solve(T, ess, n_ess, rhs.data(), kk, rel_tol, 0.0, max_iter, jacobi, s);
      st.solves++;
      st.iterations += r.iterations;
      st.max_iterations = std::max(st.max_iterations, r.iterations);
      st.converged = st.converged && r.converged;
   };
   double *kk = k.data();
   switch (type)
   {
      case 21:  // BackwardEuler
         implicit_solve(u, kk);
         kern::add_scaled(n, u, dt, kk, u, s);
         break;
      case 32:  // ImplicitMidpoint
         implicit_solve(u, kk);
         kern::add_scaled(n, u, dt, kk, u, s);
         break;
      case 22:
      case 33:  // SDIRK23
      {
         const double g = sdirk23_gamma(type);
         implicit_solve(u, kk);
         kern::add_scaled(n, u, (1. - 2. * g) * dt, kk, y.data(), s);
         kern::add_scaled(n, u, dt / 2, kk, u, s);
         implicit_solve(y.data(), kk);
         kern::add_scaled(n, u, dt / 2, kk, u, s);
         break;
      }
      case 23:  // SDIRK33
      {
         const double a = kSdirk33A, b = kSdirk33B, c = kSdirk33C;
         implicit_solve(u, kk);
         kern::add_scaled(n, u, (c - a) * dt, kk, y.data(), s);
         kern::add_scaled(n, u, b * dt, kk, u, s);
         implicit_solve(y.data(), kk);
         kern::add_scaled(n, u, (1.0 - a - b) * dt, kk, u, s);
         implicit_solve(u, kk);
         kern::add_scaled(n, u, a * dt, kk, u, s);
         break;
      }
      case 34:  // SDIRK34
      {
         const double a = sdirk34_a(), b = 1. / (6. * (2. * a - 1.) * (2. * a - 1.));
         implicit_solve(u, kk);
         kern::add_scaled(n, u, (0.5 - a) * dt, kk, y.data(), s);
         kern::add_scaled(n, u, (2. * a) * dt, kk, z.data(), s);
         kern::add_scaled(n, u, b * dt, kk, u, s);
         implicit_solve(y.data(), kk);
         kern::add_scaled(n, z.data(), (1. - 4. * a) * dt, kk, z.data(), s);
         kern::add_scaled(n, u, (1. - 2. * b) * dt, kk, u, s);
         implicit_solve(z.data(), kk);
         kern::add_scaled(n, u, b * dt, kk, u, s);
         break;
      }
      default: break;
   }
   ECM2_HIP(hipStreamSynchronize(s));
   return st;
}

} // namespace ecm2
