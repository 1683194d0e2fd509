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

#include <memory>
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
   double *xghost() { return xg_.data(); }
   double *yghost() { return yg_.data(); }
   double *recvbuf() { return rbuf_.data(); }

private:
   void rccl_exchange(bool transpose);  // P (false) or P^T (true) on the comm stream
   LocalPart part_;
   std::unique_ptr<PAForm> local_;
   DeviceArray<int> send_idx_;
   DeviceArray<double> sendbuf_, xg_, yg_, rbuf_, dl_;
   void *comm_ = nullptr;  // ncclComm_t
   hipStream_t cs_ = nullptr;
   hipEvent_t ev_pack_ = nullptr, ev_xg_ = nullptr, ev_yg_ = nullptr, ev_done_ = nullptr;
};

// In-process loopback group: all subdomains on one GPU, exchanges by device copies.
// Exercises partition, pack/unpack, split-vector kernels and interior/boundary
// ordering without RCCL (which cannot put two ranks on one device).
void par_group_mult(std::vector<ParPAForm *> &forms, const std::vector<const double *> &x,
                    const std::vector<double *> &y, hipStream_t s);
void par_group_diagonal(std::vector<ParPAForm *> &forms, const std::vector<double *> &d, hipStream_t s);

void rccl_unique_id(unsigned char *out128);

} // namespace ecm2
