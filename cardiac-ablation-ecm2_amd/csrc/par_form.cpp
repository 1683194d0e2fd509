// par_form.cpp -- see par_form.hpp.
#include "par_form.hpp"

#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>

namespace ecm2
{

#define ECM2_NCCL(call)                                                                 \
   do {                                                                                 \
      ncclResult_t r_ = (call);                                                         \
      ECM2_VERIFY(r_ == ncclSuccess, ERR_COMM, "RCCL error '" << ncclGetErrorString(r_) \
                                                      << "' in " << #call);             \
   } while (0)

void rccl_unique_id(unsigned char *out)
{
   ncclUniqueId id;
   ECM2_NCCL(ncclGetUniqueId(&id));
   static_assert(sizeof(id) == 128, "ncclUniqueId size");
   std::memcpy(out, &id, sizeof(id));
}

ParPAForm::ParPAForm(const LocalPart &part, const double *enodes_local_host, int q1d,
                     const unsigned char *rccl_id)
   : part_(part)
{
   const int nl = part.n_owned + part.n_ghost;
   local_.reset(new PAForm(part.ne_local, part.order, nl, part.gather_map.data(), q1d, part.n_owned));
   local_->set_element_nodes(enodes_local_host);
   // the Mult applies blocks [0, b_int) (interior) and [b_int, nblk) (boundary) separately
   local_->set_block_splits({part.ne_interior / kElemBlock});
   send_idx_.upload(part.send_idx);
   sendbuf_.resize(std::max<size_t>(1, part.send_idx.size()));
   rbuf_.resize(std::max<size_t>(1, part.send_idx.size()));
   xg_.resize(std::max(1, part.n_ghost));
   yg_.resize(std::max(1, part.n_ghost));
   ECM2_HIP(hipMemset(xg_.data(), 0, xg_.bytes()));
   if (rccl_id)
   {
      ncclUniqueId id;
      std::memcpy(&id, rccl_id, sizeof(id));
      ncclComm_t comm;
      ECM2_NCCL(ncclCommInitRank(&comm, part.nranks, id, part.rank));
      comm_ = comm;
   }
   // The comm stream (both transports) has the highest priority: the boundary elements and
   // the exchange kernels are dispatched ahead of the interior kernel's remaining
   // workgroups, so the exchange overlaps the interior instead of queueing behind it.
   int prio_least = 0, prio_greatest = 0;
   ECM2_HIP(hipDeviceGetStreamPriorityRange(&prio_least, &prio_greatest));
   ECM2_HIP(hipStreamCreateWithPriority(&cs_, hipStreamNonBlocking, prio_greatest));
   ECM2_HIP(hipEventCreateWithFlags(&ev_pack_, hipEventDisableTiming));
   ECM2_HIP(hipEventCreateWithFlags(&ev_xg_, hipEventDisableTiming));
   ECM2_HIP(hipEventCreateWithFlags(&ev_yg_, hipEventDisableTiming));
   ECM2_HIP(hipEventCreateWithFlags(&ev_done_, hipEventDisableTiming));
   ECM2_HIP(hipDeviceSynchronize());
}

ParPAForm::~ParPAForm()
{
   if (comm_) { (void)ncclCommDestroy((ncclComm_t)comm_); }
   if (cs_) { (void)hipStreamDestroy(cs_); }
   for (hipEvent_t e : {ev_pack_, ev_xg_, ev_yg_, ev_done_})
   {
      if (e) { (void)hipEventDestroy(e); }
   }
}

void ParPAForm::assemble(hipStream_t s) { local_->assemble(s); }

// ---------------------------------------------------------------------------------------
// Mult stages.  Per rank:
//   s  : pack (owned interface values -> send buffer), record ev_pack
//   cs : wait ev_pack; P exchange (ghost block <- owners); boundary elements; ghost shared
//        sums; record ev_yg; P^T exchange (ghost block -> owners' receive buffer); ev_done
//   s  : interior elements; wait ev_yg; owned shared sums; wait ev_done; add received
// The RCCL transport runs the stages of one rank in order; the loopback group enqueues
// them stage-major over its members, with peer device copies for the exchanges, so both
// transports share the same streams, events and overlap.
// ---------------------------------------------------------------------------------------
void ParPAForm::stage_pack(const double *x_true, double *y_true, hipStream_t s)
{
   if (!local_->use_partials())
   {
      if (part_.n_owned) { ECM2_HIP(hipMemsetAsync(y_true, 0, sizeof(double) * part_.n_owned, s)); }
      if (part_.n_ghost) { ECM2_HIP(hipMemsetAsync(yg_.data(), 0, sizeof(double) * part_.n_ghost, s)); }
   }
   kern::gather_idx((int)part_.send_idx.size(), send_idx_.data(), x_true, sendbuf_.data(), s);
   ECM2_HIP(hipEventRecord(ev_pack_, s));
   ECM2_HIP(hipStreamWaitEvent(cs_, ev_pack_, 0));
}

void ParPAForm::stage_boundary(const double *x_true, double *y_true)
{
   const int b_int = part_.ne_interior / kElemBlock;
   local_->record_start_public(cs_);
   local_->apply_blocks(x_true, xg_.data(), y_true, yg_.data(), b_int, local_->nblocks(), cs_);
   local_->record_stop_public(cs_);
   // ghost dofs are touched only by boundary elements: their sums are complete here
   local_->finish_shared(local_->n_shared_owned(), local_->n_shared(), y_true, yg_.data(), cs_);
   ECM2_HIP(hipEventRecord(ev_yg_, cs_));
}

void ParPAForm::stage_interior(const double *x_true, double *y_true, hipStream_t s)
{
   const int b_int = part_.ne_interior / kElemBlock;
   local_->record_start_public(s);
   local_->apply_blocks(x_true, xg_.data(), y_true, yg_.data(), 0, b_int, s);
   local_->record_stop_public(s);
}

void ParPAForm::stage_finish(double *y_true, hipStream_t s)
{
   ECM2_HIP(hipEventRecord(ev_done_, cs_));
   ECM2_HIP(hipStreamWaitEvent(s, ev_yg_, 0));
   local_->finish_shared(0, local_->n_shared_owned(), y_true, yg_.data(), s);
   ECM2_HIP(hipStreamWaitEvent(s, ev_done_, 0));
   kern::scatter_add_idx((int)part_.send_idx.size(), send_idx_.data(), rbuf_.data(), y_true, s);
}

void ParPAForm::rccl_exchange(bool transpose)
{
   ncclComm_t comm = (ncclComm_t)comm_;
   const int nn = (int)part_.nbrs.size();
   if (!nn) { return; }
   ECM2_NCCL(ncclGroupStart());
   for (int k = 0; k < nn; k++)
   {
      const size_t nown = part_.send_off[k + 1] - part_.send_off[k];  // my owned dofs neighbour k ghosts
      const size_t ngh = part_.recv_off[k + 1] - part_.recv_off[k];   // my ghosts owned by neighbour k
      if (!transpose)
      {
         // P (tag 41822 in the reference): owner values -> ghost copies
         if (nown) { ECM2_NCCL(ncclSend(sendbuf_.data() + part_.send_off[k], nown, ncclFloat64, part_.nbrs[k], comm, cs_)); }
         if (ngh) { ECM2_NCCL(ncclRecv(xg_.data() + part_.recv_off[k], ngh, ncclFloat64, part_.nbrs[k], comm, cs_)); }
      }
      else
      {
         // P^T (tag 41823): ghost contributions -> owners
         if (ngh) { ECM2_NCCL(ncclSend(yg_.data() + part_.recv_off[k], ngh, ncclFloat64, part_.nbrs[k], comm, cs_)); }
         if (nown) { ECM2_NCCL(ncclRecv(rbuf_.data() + part_.send_off[k], nown, ncclFloat64, part_.nbrs[k], comm, cs_)); }
      }
   }
   ECM2_NCCL(ncclGroupEnd());
}

void ParPAForm::mult(const double *x_true, double *y_true, hipStream_t s)
{
   ECM2_VERIFY(comm_, ERR_STATE, "mult needs the RCCL transport (use the loopback group otherwise)");
   stage_pack(x_true, y_true, s);
   rccl_exchange(false);
   stage_boundary(x_true, y_true);
   rccl_exchange(true);
   stage_interior(x_true, y_true, s);
   stage_finish(y_true, s);
}

void ParPAForm::diag_local(double *d_true, hipStream_t s)
{
   const int nl = part_.n_owned + part_.n_ghost;
   dl_.resize(std::max(1, nl));
   local_->assemble_diagonal(dl_.data(), s);  // local L-vector [owned | ghost]
   if (part_.n_owned)
   {
      ECM2_HIP(hipMemcpyAsync(d_true, dl_.data(), sizeof(double) * part_.n_owned, hipMemcpyDeviceToDevice, s));
   }
   if (part_.n_ghost)
   {
      ECM2_HIP(hipMemcpyAsync(yg_.data(), dl_.data() + part_.n_owned, sizeof(double) * part_.n_ghost,
                              hipMemcpyDeviceToDevice, s));
   }
}

void ParPAForm::assemble_diagonal(double *d_true, hipStream_t s)
{
   ECM2_VERIFY(comm_, ERR_STATE, "assemble_diagonal needs the RCCL transport (use the loopback group otherwise)");
   ncclComm_t comm = (ncclComm_t)comm_;
   diag_local(d_true, s);
   const int nn = (int)part_.nbrs.size();
   if (nn)
   {
      ECM2_NCCL(ncclGroupStart());
      for (int k = 0; k < nn; k++)
      {
         const size_t ns = part_.recv_off[k + 1] - part_.recv_off[k];
         const size_t nr = part_.send_off[k + 1] - part_.send_off[k];
         if (ns) { ECM2_NCCL(ncclSend(yg_.data() + part_.recv_off[k], ns, ncclFloat64, part_.nbrs[k], comm, s)); }
         if (nr) { ECM2_NCCL(ncclRecv(rbuf_.data() + part_.send_off[k], nr, ncclFloat64, part_.nbrs[k], comm, s)); }
      }
      ECM2_NCCL(ncclGroupEnd());
   }
   phase_finish(d_true, s);
}

void ParPAForm::allreduce_sum(double *dev, int n, hipStream_t s)
{
   ECM2_VERIFY(comm_, ERR_STATE, "allreduce needs the RCCL transport");
   ECM2_NCCL(ncclAllReduce(dev, dev, n, ncclFloat64, ncclSum, (ncclComm_t)comm_, s));
}

void par_group_mult(std::vector<ParPAForm *> &forms, const std::vector<const double *> &x,
                    const std::vector<double *> &y, hipStream_t s)
{
   const int n = (int)forms.size();
   ECM2_VERIFY((int)x.size() == n && (int)y.size() == n, ERR_ARG, "group size mismatch");
   for (int r = 0; r < n; r++)
   {
      ECM2_VERIFY(forms[r]->part().rank == r && forms[r]->part().nranks == n, ERR_ARG,
                  "loopback group: form " << r << " has rank " << forms[r]->part().rank);
   }
   auto slot = [&](int s_rank, int r_rank) {  // index of r_rank in s_rank's neighbour list
      const auto &nb = forms[s_rank]->part().nbrs;
      const auto it = std::find(nb.begin(), nb.end(), r_rank);
      ECM2_VERIFY(it != nb.end(), ERR_INTERNAL, "asymmetric neighbour lists");
      return (int)(it - nb.begin());
   };
   // the same stages as ParPAForm::mult, stage-major over the members; a member's
   // exchanges wait for its peers' events and copy from their buffers on its comm stream
   for (int r = 0; r < n; r++) { forms[r]->stage_pack(x[r], y[r], s); }
   for (int r = 0; r < n; r++)
   {
      ParPAForm &f = *forms[r];
      const LocalPart &pr = f.part();
      for (size_t k = 0; k < pr.nbrs.size(); k++)
      {
         const int o = pr.nbrs[k], j = slot(o, r);
         const LocalPart &po = forms[o]->part();
         const size_t cnt = pr.recv_off[k + 1] - pr.recv_off[k];
         ECM2_VERIFY(cnt == (size_t)(po.send_off[j + 1] - po.send_off[j]), ERR_INTERNAL,
                     "exchange size mismatch " << r << "<-" << o);
         if (!cnt) { continue; }
         ECM2_HIP(hipStreamWaitEvent(f.comm_stream(), forms[o]->event_packed(), 0));
         ECM2_HIP(hipMemcpyAsync(f.xghost() + pr.recv_off[k], forms[o]->sendbuf() + po.send_off[j],
                                 cnt * sizeof(double), hipMemcpyDeviceToDevice, f.comm_stream()));
      }
   }
   for (int r = 0; r < n; r++) { forms[r]->stage_boundary(x[r], y[r]); }
   for (int r = 0; r < n; r++)
   {
      ParPAForm &f = *forms[r];
      const LocalPart &pr = f.part();
      for (size_t k = 0; k < pr.nbrs.size(); k++)
      {
         const int g = pr.nbrs[k], j = slot(g, r);
         const LocalPart &pg = forms[g]->part();
         const size_t cnt = pr.send_off[k + 1] - pr.send_off[k];
         ECM2_VERIFY(cnt == (size_t)(pg.recv_off[j + 1] - pg.recv_off[j]), ERR_INTERNAL,
                     "reduce size mismatch " << r << "<-" << g);
         if (!cnt) { continue; }
         ECM2_HIP(hipStreamWaitEvent(f.comm_stream(), forms[g]->event_ghosts_summed(), 0));
         ECM2_HIP(hipMemcpyAsync(f.recvbuf() + pr.send_off[k], forms[g]->yghost() + pg.recv_off[j],
                                 cnt * sizeof(double), hipMemcpyDeviceToDevice, f.comm_stream()));
      }
   }
   for (int r = 0; r < n; r++) { forms[r]->stage_interior(x[r], y[r], s); }
   for (int r = 0; r < n; r++) { forms[r]->stage_finish(y[r], s); }
}

} // namespace ecm2

namespace ecm2
{
// P^T of the loopback group: every member's ghost block (yghost) copied into its owner's
// receive buffer, then added into the owner's true vector.
static void group_reduce_ghosts(std::vector<ParPAForm *> &forms, const std::vector<double *> &y, hipStream_t s)
{
   const int n = (int)forms.size();
   for (int r = 0; r < n; r++)
   {
      const LocalPart &pr = forms[r]->part();
      for (size_t k = 0; k < pr.nbrs.size(); k++)
      {
         const int g = pr.nbrs[k];
         const auto &nb = forms[g]->part().nbrs;
         const int j = (int)(std::find(nb.begin(), nb.end(), r) - nb.begin());
         ECM2_VERIFY(j < (int)nb.size(), ERR_INTERNAL, "asymmetric neighbour lists");
         const LocalPart &pg = forms[g]->part();
         const size_t cnt = pr.send_off[k + 1] - pr.send_off[k];
         if (cnt)
         {
            ECM2_HIP(hipMemcpyAsync(forms[r]->recvbuf() + pr.send_off[k], forms[g]->yghost() + pg.recv_off[j],
                                    cnt * sizeof(double), hipMemcpyDeviceToDevice, s));
         }
      }
   }
   for (int r = 0; r < n; r++) { forms[r]->phase_finish(y[r], s); }
}

void par_group_diagonal(std::vector<ParPAForm *> &forms, const std::vector<double *> &d, hipStream_t s)
{
   ECM2_VERIFY(d.size() == forms.size(), ERR_ARG, "group size mismatch");
   for (size_t r = 0; r < forms.size(); r++) { forms[r]->diag_local(d[r], s); }
   group_reduce_ghosts(forms, d, s);
}
} // namespace ecm2
