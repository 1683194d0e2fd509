// par_form.hpp -- distributed PA form: y_true = P^T A_local P x_true over RCCL (xGMI).
//
// Reference: ParBilinearForm (fem/pbilinearform.cpp:475-511) -> RAPOperator(P, A, P)
// (linalg/operator.hpp:959-977) with P = DeviceConformingProlongationOperator
// (fem/pfespace.cpp:5259-5532): pack (BcastBeginCopy :5340-5360), MPI_Isend/Irecv
// tag 41822 (:5412-5437), unpack; P^T: pack ghosts, MPI tag 41823 (:5504-5529),
// ReduceEndAssemble (:5468-5494).
//
// MI355X design: one process per GPU; the local L-vector is [owned | ghost] so P is
// "receive the ghost block in place" and P^T is "send the ghost block in place, add
// what arrives into the owned interface dofs"; each exchange is one grouped
// ncclSend/ncclRecv over the partition's exchange schedule (partition.hpp) on a dedicated
// comm stream, overlapped with the interior elements (those touching no ghost dof), which
// are enqueued before the boundary ones.
#pragma once

#include "pa_form.hpp"
#include "partition.hpp"

#include <map>
#include <memory>
#include <utility>
#include <vector>

namespace ecm2
{

class ParPAForm
{
public:
   // rccl_id: 128-byte ncclUniqueId shared by all ranks (RCCL transport), or null for a
   // member of an in-process loopback group (par_group_mult).
   ParPAForm(const LocalPart &part, const double *enodes_local_host, int q1d,
             const unsigned char *rccl_id);
   ~ParPAForm();

   PAForm &local() { return *local_; }
   const PAForm &local() const { return *local_; }
   const LocalPart &part() const { return part_; }
   int true_size() const { return part_.n_owned; }

   void assemble(hipStream_t s);
   size_t algorithmic_bytes() const;
   // y_true = P^T A P x_true (RCCL transport).
   void mult(const double *x_true, double *y_true, hipStream_t s);
   // Diagonal of P^T A P on the true dofs: local PA diagonal, ghost entries summed into
   // their owners (ParBilinearForm::AssembleDiagonal -> P^T d_local, pbilinearform.cpp).
   void assemble_diagonal(double *d_true, hipStream_t s);
   // In-place sum over ranks of n device doubles (the dots of the parallel PCG).
   void allreduce_sum(double *dev, int n, hipStream_t s);
   // Pieces of assemble_diagonal shared with the loopback group.
   void diag_local(double *d_true, hipStream_t s);  // d_true = owned part, ghost part -> yghost()

   // Mult stages, shared by the RCCL transport and the loopback group.
   void stage_pack(const double *x_true, double *y_true, hipStream_t s);
   void stage_boundary(const double *x_true, double *y_true);   // on the comm stream
   void stage_interior(const double *x_true, double *y_true, hipStream_t s);
   void stage_finish(double *y_true, hipStream_t s);
   void phase_finish(double *y_true, hipStream_t s)  // add the received P^T contributions
   {
      kern::scatter_add_idx((int)part_.send_idx.size(), send_idx_.data(), rbuf_.data(), y_true, s);
   }
   // Serial schedule (one stream): pack, the P exchange, ONE apply launch over every local
   // block, [RAP: ghost sums, P^T exchange], the shared-dof sums.  The overlapped schedule runs
   // the interior beside the exchange + boundary elements on the comm stream instead.
   bool serial() const { return serial_; }
   // Schedule of the Mult (serial: true, overlapped: false) and its launch form (graph: 1
   // captured HIP graph, 0 direct launches, -1 the schedule's default); before Assemble.
   void set_schedule(bool serial, int graph);
   void stage_serial_apply(const double *x_true, double *y_true, hipStream_t s);
   hipStream_t comm_stream() const { return cs_; }
   bool pack_needed() const { return pack_needed_; }
   const int *send_idx_data() const { return send_idx_.data(); }
   double *sendbuf_data() { return sendbuf_.data(); }
   double *yghost() { return yg_.data(); }
   hipEvent_t event_packed() const { return ev_pack_; }
   hipEvent_t event_ghosts_summed() const { return ev_yg_; }

   // The exchange schedule of P / P^T (exchange_schedule) and the device address of one
   // transfer's data (x_true: the true vector of the Mult being enqueued).
   const std::vector<Xfer> &schedule(bool transpose) const { return transpose ? sched_t_ : sched_p_; }
   double *xfer_ptr(const Xfer &t, const double *x_true);
   // The x of the last loopback-group Mult and the local form's assembly it ran on: a member's
   // RAP rows copy the state it left (par_group_mult_member checks it is current).
   void note_group_mult(const double *x_true) { group_x_ = x_true; group_gen_ = local_->generation(); }
   bool group_mult_current(const double *x_true) const
   {
      return group_x_ == x_true && group_gen_ == local_->generation();
   }

private:
   void rccl_exchange(bool transpose, const double *x_true, hipStream_t st);  // grouped send/recv on st
   void mult_stages(const double *x_true, double *y_true, hipStream_t s);
   int b_int() const { return part_.ne_interior / kElemBlock; }
   void drop_graphs();
   LocalPart part_;
   std::unique_ptr<PAForm> local_;
   std::vector<Xfer> sched_p_, sched_t_;
   bool pack_needed_ = false;           // some P send goes through the packed buffer
   bool serial_ = true;                 // serial schedule (serial())
   int graph_mode_ = -1;                // set_schedule
   DeviceArray<int> send_idx_;
   DeviceArray<double> sendbuf_, xg_, yg_, rbuf_, dl_;
   void *comm_ = nullptr;               // ncclComm_t
   hipStream_t cs_ = nullptr;           // comm stream (highest priority)
   hipEvent_t ev_pack_ = nullptr, ev_xg_ = nullptr, ev_yg_ = nullptr, ev_done_ = nullptr;
   // The Mult as a HIP graph per (x, y) pair: one launch instead of ~15 API calls.  A graph
   // bakes in the local form's buffers and kernels, so the cache belongs to one assembly of
   // it (generation) and holds at most kMaxGraphs entries.
   static constexpr size_t kMaxGraphs = 4;
   hipStream_t cap_ = nullptr;          // capture stream
   std::map<std::pair<const double *, double *>, hipGraphExec_t> graphs_;
   long graph_gen_ = -1;
   bool graph_failed_ = false;
   bool p2p_warm_ = false;  // one direct Mult ran (RCCL peer connections exist) before any capture
   const double *group_x_ = nullptr;  // note_group_mult
   long group_gen_ = -1;
};

// RCCL point-to-point self-test (one-rank communicator, direct or graph-captured): max error.
double rccl_p2p_selftest(bool graph, int n);

// In-process loopback group: all subdomains on one GPU, exchanges by device copies that
// follow the members' exchange schedules (each receive copies the peer's matching send).
// Exercises partition, schedule, split-vector kernels and interior/boundary ordering without
// RCCL (which cannot put two ranks on one device).
// rccl_self: the exchanges go through RCCL instead of device copies -- a one-rank communicator
// sends each schedule row to itself and receives it into the peer's row (grouped ncclSend /
// ncclRecv on s, capturable in a HIP graph); serial schedule only.
void par_group_mult(std::vector<ParPAForm *> &forms, const std::vector<const double *> &x,
                    const std::vector<double *> &y, hipStream_t s, bool rccl_self = false);
void par_group_diagonal(std::vector<ParPAForm *> &forms, const std::vector<double *> &d, hipStream_t s);
// One member's rows of the group operator, y[r] = (A x)_r: member r's stages alone, exactly as
// one rank of the RCCL transport runs them (interior on s, exchange + boundary on r's comm
// stream, then the summation), its ghost values copied from the peers' x (or, for packed sends,
// their send buffers as the last group Mult left them).  RAP (serial schedule): + the ghost sums
// and the P^T receive, copied from the peers' y ghost blocks as the last group Mult left them.
// The other members' y are not touched.  This is what a rank's Mult costs on its own GPU, short
// of the xGMI transfer time.  Run one group Mult on the same x arrays first: RAP and packed sends
// fail with ERR_STATE when the peers' last group Mult ran on other x arrays or another assembly.
// In-place sum of n device scalars on the one-rank RCCL communicator of the self transport: the
// collective call a rank's solver makes, without the peers (member emulation, MemberOp).
void group_self_allreduce(double *dev, int n, hipStream_t s);
void par_group_mult_member(std::vector<ParPAForm *> &forms, const std::vector<const double *> &x,
                           const std::vector<double *> &y, int r, hipStream_t s);

void rccl_unique_id(unsigned char *out128);

} // namespace ecm2
