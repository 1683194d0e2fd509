// solvers.hpp -- the callers of the PA operator: constrained Jacobi-PCG and the SDIRK
// time steppers of an ex16-style conduction (Pennes bioheat) operator, all device
// resident, over one operator interface that the serial form, the RCCL-distributed form
// and the in-process loopback group implement.
//
// Reference:
//   Operator (the solver-facing interface)     linalg/operator.hpp:24-110
//   ConstrainedOperator DIAG_ONE               linalg/operator.cpp:586-646
//   CGSolver::Mult                             linalg/solvers.cpp:869-1004
//   OperatorJacobiSmoother (PA diagonal)       linalg/solvers.hpp:421, bilinearform_ext.cpp:370-454
//   parallel dot (MPI_Allreduce)               linalg/hypre / InnerProduct(comm, ...)
//   BackwardEuler / SDIRK23 / SDIRK33 / ImplicitMidpoint / SDIRK34 ::Step
//                                              linalg/ode.cpp:682-859, selection :77-91
//   ConductionOperator::ImplicitSolve          examples/ex16.cpp:327-354
#pragma once

#include "pa_form.hpp"
#include "par_form.hpp"

#include <vector>

namespace ecm2
{

// A square operator on this rank's slice of the true-dof vector.
class LinOp
{
public:
   virtual ~LinOp() = default;
   virtual int size() const = 0;
   // y = A x (Operator::Mult; y overwritten)
   virtual void mult(const double *x, double *y, hipStream_t s) = 0;
   // diagonal of the global operator on this rank's true dofs
   virtual void diagonal(double *d, hipStream_t s) = 0;
   // in-place global sum of n device scalars over all ranks (serial: nothing to do)
   virtual void sum_scalars(double *dev, int n, hipStream_t s) { (void)dev; (void)n; (void)s; }
   // true when sum_scalars communicates (a locally reduced scalar is not yet global)
   virtual bool distributed() const { return false; }
   // The Mult with its energy x^T A x folded in as energy_parts() partials (PAForm::mult_energy),
   // or 0 when this operator does not fold it
   virtual int energy_parts() const { return 0; }
   virtual void mult_energy(const double *x, double *y, double *en, hipStream_t s)
   {
      (void)x; (void)y; (void)en; (void)s;
      ECM2_VERIFY(false, ERR_UNSUPPORTED, "this operator does not fold the Mult's energy");
   }
};

class FormOp : public LinOp
{
public:
   explicit FormOp(PAForm &f) : f_(f) {}
   int size() const override { return f_.ndofs(); }
   void mult(const double *x, double *y, hipStream_t s) override { f_.mult(x, y, s); }
   void diagonal(double *d, hipStream_t s) override { f_.assemble_diagonal(d, s); }
   int energy_parts() const override { return f_.energy_parts(); }
   void mult_energy(const double *x, double *y, double *en, hipStream_t s) override { f_.mult_energy(x, y, en, s); }

private:
   PAForm &f_;
};

class ParFormOp : public LinOp
{
public:
   explicit ParFormOp(ParPAForm &f) : f_(f) {}
   int size() const override { return f_.true_size(); }
   void mult(const double *x, double *y, hipStream_t s) override { f_.mult(x, y, s); }
   void diagonal(double *d, hipStream_t s) override { f_.assemble_diagonal(d, s); }
   void sum_scalars(double *dev, int n, hipStream_t s) override { f_.allreduce_sum(dev, n, s); }
   bool distributed() const override { return true; }

private:
   ParPAForm &f_;
};

// The loopback group as one operator on the concatenated true vectors of its members
// (rank r's slice at offset(r)); dots over the concatenation are already global.
class GroupOp : public LinOp
{
public:
   explicit GroupOp(std::vector<ParPAForm *> forms);
   int size() const override { return n_; }
   void mult(const double *x, double *y, hipStream_t s) override;
   void diagonal(double *d, hipStream_t s) override;
   int offset(int r) const { return off_[r]; }

private:
   std::vector<ParPAForm *> forms_;
   std::vector<int> off_;
   int n_ = 0;
};

// One member of the loopback group as one rank's operator (measurement of a rank's solver
// iteration on its own GPU; no reference counterpart): Mult = par_group_mult_member (the P
// exchange as device copies from the peers' x, held in a private concatenated vector), the
// dots summed by a real ncclAllReduce on a one-rank communicator (the collective call without
// the xGMI hops).  Vectors are the member's true dofs.
class MemberOp : public LinOp
{
public:
   MemberOp(std::vector<ParPAForm *> forms, int member);
   int size() const override { return forms_[member_]->true_size(); }
   void mult(const double *x, double *y, hipStream_t s) override;
   void diagonal(double *d, hipStream_t s) override;
   void sum_scalars(double *dev, int n, hipStream_t s) override { group_self_allreduce(dev, n, s); }
   bool distributed() const override { return true; }

private:
   std::vector<ParPAForm *> forms_;
   int member_;
   std::vector<int> off_;
   DeviceArray<double> peers_, yscratch_;  // the peers' x (zeros) and y (never read), concatenated
};

struct PCGResult
{
   int iterations = 0;
   double final_norm = 0.0, initial_norm = 0.0;
   bool converged = false;
};

// Constrained (DIAG_ONE on ess) Jacobi-PCG, x overwritten (iterative_mode = false).
// Scalars stay on the device; one 8-byte read-back per iteration for the stopping test.
PCGResult pcg_solve(LinOp &A, const int *ess_dev, int n_ess, const double *b, double *x,
                    double rel_tol, double abs_tol, int max_iter, bool jacobi, hipStream_t s);
PCGResult pcg_solve(PAForm &A, const int *ess_dev, int n_ess, const double *b, double *x,
                    double rel_tol, double abs_tol, int max_iter, bool jacobi, hipStream_t s);

// ODESolver::SelectImplicit numbering (ode.cpp:77-91): 21 BackwardEuler, 22 SDIRK23(L-stable),
// 23 SDIRK33, 32 ImplicitMidpoint, 33 SDIRK23 (A-stable, order 3), 34 SDIRK34.
bool ode_implicit_supported(int type);
// The implicit coefficient c of every stage solve (M + c*dt*K) k = -K u of `type`.
double ode_implicit_coeff(int type);

struct StepStats
{
   int solves = 0, iterations = 0, max_iterations = 0;
   bool converged = true;
};

// One implicit step u <- u(t + dt) of M du/dt = -K u (ex16 ConductionOperator, slope
// form): each stage solves T k = -K u_stage with T = M + c*dt*K supplied assembled by
// the caller (c = ode_implicit_coeff(type)); ess dofs keep their values (k = 0 there).
StepStats ode_step(int type, LinOp &T, LinOp &K, double dt, double *u, const int *ess_dev, int n_ess,
                   double rel_tol, int max_iter, bool jacobi, hipStream_t s);

} // namespace ecm2
