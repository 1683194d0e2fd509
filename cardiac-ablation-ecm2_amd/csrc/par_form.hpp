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
// what arrives into the owned interface dofs"; the exchange is one grouped
// ncclSend/ncclRecv per direction on a dedicated comm stream, overlapped with the
// interior elements (those touching no ghost dof), which run before the boundary ones.
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
   // member of an in-process loopback group (ParGroup).
   ParPAForm(const LocalPart &part, const double *enodes_local_host, int q1d,
             const unsigned char *rccl_id);
   ~ParPAForm();

   PAForm &local() { return *local_; }
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

   // Mult stages (par_form.cpp), shared by the RCCL transport and the loopback group.
   void stage_pack(const double *x_true, double *y_true, hipStream_t s);
   void stage_boundary(const double *x_true, double *y_true);   // on the comm stream
   void stage_interior(const double *x_true, double *y_true, hipStream_t s);
   void stage_finish(double *y_true, hipStream_t s);
   void phase_finish(double *y_true, hipStream_t s)  // add the received P^T contributions
   {
      kern::scatter_add_idx((int)part_.send_idx.size(), send_idx_.data(), rbuf_.data(), y_true, s);
   }
   hipStream_t comm_stream() const { return cs_; }
   hipEvent_t event_packed() const { return ev_pack_; }
   hipEvent_t event_ghosts_summed() const { return ev_yg_; }

   // buffers (device)
   double *sendbuf() { return sendbuf_.data(); }
   // P send buffer of neighbour slot k: x_true itself where the rank's owned dofs that
   // neighbour k ghosts form one contiguous range (z-slabs: the top dof planes), else the
   // packed buffer.
   const double *send_ptr(int k, const double *x_true) const
   {
      return send_start_[k] >= 0 ? x_true + send_start_[k] : sendbuf_.data() + part_.send_off[k];
   }
   double *xghost() { return xg_.data(); }
   double *yghost() { return yg_.data(); }
   double *recvbuf() { return rbuf_.data(); }

private:
   void rccl_exchange(bool transpose);  // P (false) or P^T (true) on the comm stream
   void mult_stages(const double *x_true, double *y_true, hipStream_t s, bool emu);
   int b_int() const { return part_.ne_interior / kElemBlock; }
   int b_split_ = 0;                    // interior part A = [0, b_split_) (0: no split)
   std::vector<int> send_start_;        // per neighbour: first owned index of a contiguous send range, or -1
   bool pack_needed_ = true;            // some neighbour's send range is not contiguous
   const double *x_cur_ = nullptr;      // x_true of the Mult being enqueued (contiguous sends)
   hipEvent_t ev_bnd_ = nullptr;        // boundary elements applied (comm stream)
   // Mult as a HIP graph per (x, y) pair: one launch instead of ~15 API calls
   hipStream_t cap_ = nullptr;          // capture stream
   std::map<std::pair<const double *, double *>, hipGraphExec_t> graphs_;
   bool graph_failed_ = false;
   bool p2p_warm_ = false;  // one direct Mult ran (RCCL peer connections exist) before any capture
   LocalPart part_;
   std::unique_ptr<PAForm> local_;
   DeviceArray<int> send_idx_;
   DeviceArray<double> sendbuf_, xg_, yg_, rbuf_, dl_;
   void *comm_ = nullptr;  // ncclComm_t
   void self_exchange(bool transpose);  // ECM2_EMULATE_EXCHANGE measurement aid
   hipStream_t cs_ = nullptr;
   hipStream_t is_ = nullptr;       // interior stream, CU-masked against cs_ (null: interior on the caller's stream)
   hipEvent_t ev_s_ = nullptr, ev_int_ = nullptr;
   hipEvent_t ev_pack_ = nullptr, ev_xg_ = nullptr, ev_yg_ = nullptr, ev_done_ = nullptr;
};

// RCCL point-to-point self-test (one-rank communicator, direct or graph-captured): max error.
double rccl_p2p_selftest(bool graph, int n);

// In-process loopback group: all subdomains on one GPU, exchanges by device copies.
// Exercises partition, pack/unpack, split-vector kernels and interior/boundary
// ordering without RCCL (which cannot put two ranks on one device).
void par_group_mult(std::vector<ParPAForm *> &forms, const std::vector<const double *> &x,
                    const std::vector<double *> &y, hipStream_t s);
void par_group_diagonal(std::vector<ParPAForm *> &forms, const std::vector<double *> &d, hipStream_t s);

void rccl_unique_id(unsigned char *out128);

} // namespace ecm2
