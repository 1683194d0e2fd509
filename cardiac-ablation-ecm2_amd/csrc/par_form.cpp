// par_form.cpp -- see par_form.hpp.
#include "par_form.hpp"

#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>

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

// Transport self-test: a one-rank communicator exchanging n doubles with itself through
// grouped ncclSend/ncclRecv, launched directly or captured in a HIP graph and replayed
// three times (the form's graph-captured Mult relies on RCCL point-to-point capture).
double rccl_p2p_selftest(bool graph, int n)
{
   ncclUniqueId id;
   ECM2_NCCL(ncclGetUniqueId(&id));
   ncclComm_t comm;
   ECM2_NCCL(ncclCommInitRank(&comm, 1, id, 0));
   hipStream_t st;
   ECM2_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
   DeviceArray<double> a, b;
   a.resize(std::max(1, n));
   b.resize(std::max(1, n));
   std::vector<double> h(std::max(1, n));
   double err = 0.0;
   hipGraphExec_t ge = nullptr;
   for (int rep = 0; rep < 3; rep++)
   {
      for (int i = 0; i < n; i++) { h[i] = 0.5 * i + rep; }
      // on st: a non-blocking stream does not order itself after the null stream's memset
      ECM2_HIP(hipMemcpyAsync(a.data(), h.data(), sizeof(double) * n, hipMemcpyHostToDevice, st));
      ECM2_HIP(hipMemsetAsync(b.data(), 0, sizeof(double) * n, st));
      auto exchange = [&] {
         ECM2_NCCL(ncclGroupStart());
         ECM2_NCCL(ncclSend(a.data(), n, ncclFloat64, 0, comm, st));
         ECM2_NCCL(ncclRecv(b.data(), n, ncclFloat64, 0, comm, st));
         ECM2_NCCL(ncclGroupEnd());
      };
      if (graph)
      {
         if (rep == 0)
         {
            hipGraph_t g = nullptr;
            ECM2_HIP(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
            exchange();
            ECM2_HIP(hipStreamEndCapture(st, &g));
            ECM2_HIP(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
            ECM2_HIP(hipGraphDestroy(g));
         }
         ECM2_HIP(hipGraphLaunch(ge, st));
      }
      else { exchange(); }
      ECM2_HIP(hipStreamSynchronize(st));
      std::vector<double> r(std::max(1, n));
      ECM2_HIP(hipMemcpyAsync(r.data(), b.data(), sizeof(double) * n, hipMemcpyDeviceToHost, st));
      ECM2_HIP(hipStreamSynchronize(st));
      for (int i = 0; i < n; i++) { err = std::max(err, std::fabs(r[i] - h[i])); }
      if (graph && rep == 2) { ECM2_HIP(hipGraphExecDestroy(ge)); ge = nullptr; }
   }
   ECM2_HIP(hipStreamDestroy(st));
   (void)ncclCommDestroy(comm);
   return err;
}

// The distributed Mult as one captured HIP graph (per (x, y) pair) or as direct launches.
// The serial schedule is ~5 API calls per Mult, fewer host-microseconds than its GPU time even
// at C4 / 8 ranks, and a graph replay leaves ~9 us between consecutive Mults
// (profiles/r2_member_emul.txt): direct launches.  The overlapped schedule's ~15 calls (event
// pairs for the comm stream) are host-bound without the graph.  ECM2_PAR_GRAPH=0 / 1 forces
// either (the operator is the same).
static bool par_graph(bool serial, int mode)
{
   static const int v = [] {
      const char *e = std::getenv("ECM2_PAR_GRAPH");
      return e ? (std::string(e) == "0" ? 0 : 1) : -1;
   }();
   if (mode >= 0) { return mode == 1; }
   return v < 0 ? !serial : v == 1;
}

ParPAForm::ParPAForm(const LocalPart &part, const double *enodes_local_host, int q1d,
                     const unsigned char *rccl_id)
   : part_(part)
{
   const int nl = part.n_owned + part.n_ghost;
   local_.reset(new PAForm(part.ne_local, part.order, nl, part.gather_map.data(), q1d, part.n_owned));
   local_->set_element_nodes(enodes_local_host);
   // Mult schedule: serial by default (set_schedule; the overlapped one applies blocks [0,
   // b_int) (interior) beside the exchange and [b_int, nblk) (boundary, with the
   // one-block-per-workgroup latency kernel) on the comm stream -- profiles/r2_member_trace.txt:
   // the interior kernel takes every CU slot and the boundary kernel beside it ends with it)
   set_schedule(true, -1);
   sched_p_ = exchange_schedule(part, false);
   sched_t_ = exchange_schedule(part, true);
   for (const Xfer &t : sched_p_) { pack_needed_ |= t.buf == XBUF_SENDBUF; }
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

void ParPAForm::set_schedule(bool serial, int graph)
{
   ECM2_VERIFY(graph >= -1 && graph <= 1, ERR_ARG, "graph mode " << graph << " not in {-1, 0, 1}");
   serial_ = serial;
   graph_mode_ = graph;
   drop_graphs();
   const int bi = part_.ne_interior / kElemBlock;
   if (!serial_)
   {
      local_->set_block_splits({bi});
      local_->set_latency_from(bi);
   }
   else
   {
      // one launch over every block, but the element order is still derived per segment
      // [interior | boundary]: the interior's face-linked bricks are anchored at its own first
      // layer, so none of them touches a ghost dof and all are lattice-addressed (anchored at the
      // local mesh's first layer, the bricks of the ghost-touching bottom layer read the map).
      // A split on a multiple of 4 blocks keeps the plan's workgroups (4 blocks from each
      // segment's start) those of the single launch.
      local_->set_block_splits({bi / 4 * 4});
      local_->set_latency_from(-1);
   }
}

void ParPAForm::drop_graphs()
{
   for (auto &kv : graphs_) { (void)hipGraphExecDestroy(kv.second); }
   graphs_.clear();
}

ParPAForm::~ParPAForm()
{
   drop_graphs();
   if (comm_) { (void)ncclCommDestroy((ncclComm_t)comm_); }
   if (cs_) { (void)hipStreamDestroy(cs_); }
   if (cap_) { (void)hipStreamDestroy(cap_); }
   for (hipEvent_t e : {ev_pack_, ev_xg_, ev_yg_, ev_done_})
   {
      if (e) { (void)hipEventDestroy(e); }
   }
}

void ParPAForm::assemble(hipStream_t s)
{
   drop_graphs();  // the local form's buffers and kernel may change
   local_->assemble(s);
}

size_t ParPAForm::algorithmic_bytes() const
{
   // SURVEY §8(d) over the rank's own elements and true dofs (OVERLAP's ghost elements are
   // duplicated work, not counted)
   const PAForm &f = *local_;
   const size_t nq = (size_t)f.q1d() * f.q1d() * f.q1d(), nd = (size_t)f.d1d() * f.d1d() * f.d1d();
   const size_t nc = (f.has_diffusion() ? 6 : 0) + (f.has_mass() ? 1 : 0);
   return 8ull * part_.ne_owned * nq * nc + 16ull * part_.n_owned + 4ull * part_.ne_owned * nd;
}

double *ParPAForm::xfer_ptr(const Xfer &t, const double *x_true)
{
   switch (t.buf)
   {
      case XBUF_X_TRUE: return const_cast<double *>(x_true) + t.off;
      case XBUF_SENDBUF: return sendbuf_.data() + t.off;
      case XBUF_XGHOST: return xg_.data() + t.off;
      case XBUF_YGHOST: return yg_.data() + t.off;
      case XBUF_RECVBUF: return rbuf_.data() + t.off;
   }
   ECM2_VERIFY(false, ERR_INTERNAL, "unknown exchange buffer " << t.buf);
}

// ---------------------------------------------------------------------------------------
// Mult stages.  Per rank:
//   s  : record ev_xg (x ready)
//   cs : wait ev_xg; pack (owned interface values -> send buffer) if a send needs it; ev_pack
//   s  : interior elements (enqueued first: whatever is enqueued first starts first)
//   cs : P exchange (ghost block <- owners); boundary elements; [RAP: ghost shared sums,
//        ev_yg, P^T exchange (ghost block -> owners' receive buffer)]; ev_done
//   s  : wait ev_done; owned shared sums [RAP: + the received contributions]
// The RCCL transport runs the stages of one rank in order; the loopback group enqueues
// them stage-major over its members with device copies for the exchanges, so both
// transports share the same streams, events and overlap.
// ---------------------------------------------------------------------------------------
void ParPAForm::stage_pack(const double *x_true, double *y_true, hipStream_t s)
{
   if (!local_->use_partials())
   {
      if (part_.n_owned) { ECM2_HIP(hipMemsetAsync(y_true, 0, sizeof(double) * part_.n_owned, s)); }
      if (part_.n_ghost) { ECM2_HIP(hipMemsetAsync(yg_.data(), 0, sizeof(double) * part_.n_ghost, s)); }
   }
   // the comm stream picks up x (and the memsets) from s, then packs on its own: the
   // interior kernel on s does not queue behind the pack
   ECM2_HIP(hipEventRecord(ev_xg_, s));
   ECM2_HIP(hipStreamWaitEvent(cs_, ev_xg_, 0));
   if (pack_needed_)
   {
      kern::gather_idx((int)part_.send_idx.size(), send_idx_.data(), x_true, sendbuf_.data(), cs_);
   }
   ECM2_HIP(hipEventRecord(ev_pack_, cs_));
}

void ParPAForm::stage_boundary(const double *x_true, double *y_true)
{
   local_->record_start_public(cs_);
   local_->apply_blocks(x_true, xg_.data(), y_true, yg_.data(), b_int(), local_->nblocks(), cs_, true);
   local_->record_stop_public(cs_);
   // ghost dofs are touched only by boundary elements: their sums are complete here (OVERLAP:
   // the ghost outputs are discarded, nothing to sum)
   if (!part_.overlap) { local_->finish_shared(local_->n_shared_owned(), local_->n_shared(), y_true, yg_.data(), cs_); }
   ECM2_HIP(hipEventRecord(ev_yg_, cs_));
}

void ParPAForm::stage_interior(const double *x_true, double *y_true, hipStream_t s)
{
   local_->record_start_public(s);
   local_->apply_blocks(x_true, xg_.data(), y_true, yg_.data(), 0, b_int(), s);
   local_->record_stop_public(s);
}

void ParPAForm::stage_finish(double *y_true, hipStream_t s)
{
   ECM2_HIP(hipEventRecord(ev_done_, cs_));
   ECM2_HIP(hipStreamWaitEvent(s, ev_done_, 0));
   local_->finish_shared(0, local_->n_shared_owned(), y_true, yg_.data(), s);
   // OVERLAP: every contribution to an owned dof was computed here; RAP: add what the
   // neighbours' ghost copies contributed (P^T)
   if (!part_.overlap) { phase_finish(y_true, s); }
}

void ParPAForm::rccl_exchange(bool transpose, const double *x_true, hipStream_t st)
{
   ncclComm_t comm = (ncclComm_t)comm_;
   const std::vector<Xfer> &sch = schedule(transpose);
   if (sch.empty()) { return; }
   ECM2_NCCL(ncclGroupStart());
   for (const Xfer &t : sch)
   {
      double *p = xfer_ptr(t, x_true);
      if (t.send) { ECM2_NCCL(ncclSend(p, t.count, ncclFloat64, t.peer, comm, st)); }
      else { ECM2_NCCL(ncclRecv(p, t.count, ncclFloat64, t.peer, comm, st)); }
   }
   ECM2_NCCL(ncclGroupEnd());
}

// Serial schedule, after the P exchange on s: every local block in one launch, then [RAP: the
// ghost dofs' sums (sent by the caller's P^T exchange)] -- no comm stream, no cross-stream
// event: the interior kernel would otherwise occupy every CU slot and the boundary kernel
// beside it finishes only with it (profiles/r2_member_trace.txt).
void ParPAForm::stage_serial_apply(const double *x_true, double *y_true, hipStream_t s)
{
   if (!local_->use_partials())
   {
      if (part_.n_owned) { ECM2_HIP(hipMemsetAsync(y_true, 0, sizeof(double) * part_.n_owned, s)); }
      if (part_.n_ghost) { ECM2_HIP(hipMemsetAsync(yg_.data(), 0, sizeof(double) * part_.n_ghost, s)); }
   }
   local_->record_start_public(s);
   local_->apply_blocks(x_true, xg_.data(), y_true, yg_.data(), 0, local_->nblocks(), s);
   local_->record_stop_public(s);
   if (!part_.overlap) { local_->finish_shared(local_->n_shared_owned(), local_->n_shared(), y_true, yg_.data(), s); }
}

void ParPAForm::mult_stages(const double *x_true, double *y_true, hipStream_t s)
{
   if (serial_)
   {
      if (pack_needed_) { kern::gather_idx((int)part_.send_idx.size(), send_idx_.data(), x_true, sendbuf_.data(), s); }
      rccl_exchange(false, x_true, s);
      stage_serial_apply(x_true, y_true, s);
      if (!part_.overlap) { rccl_exchange(true, x_true, s); }
      local_->finish_shared(0, local_->n_shared_owned(), y_true, yg_.data(), s);
      if (!part_.overlap) { phase_finish(y_true, s); }
      return;
   }
   stage_pack(x_true, y_true, s);
   stage_interior(x_true, y_true, s);
   rccl_exchange(false, x_true, cs_);
   stage_boundary(x_true, y_true);
   if (!part_.overlap) { rccl_exchange(true, x_true, cs_); }
   stage_finish(y_true, s);
}

void ParPAForm::mult(const double *x_true, double *y_true, hipStream_t s)
{
   ECM2_VERIFY(comm_, ERR_STATE, "mult needs the RCCL transport (use the loopback group otherwise)");
   ECM2_VERIFY(local_->assembled(), ERR_STATE, "Mult before Assemble");
   if (graph_gen_ != local_->generation())
   {
      drop_graphs();  // the cached graphs bake in the previous assembly's buffers and kernels
      graph_gen_ = local_->generation();
   }
   if (!par_graph(serial_, graph_mode_) || graph_failed_ || local_->timing_on() || !p2p_warm_)
   {
      // the first Mult runs directly on every rank: RCCL sets up its peer connections
      // lazily at the first send/recv, which then happens outside a stream capture
      mult_stages(x_true, y_true, s);
      p2p_warm_ = true;
      return;
   }
   // One HIP graph per (x, y): the ~15 launches / event operations / RCCL group calls of a
   // Mult cost more host time than the GPU work at 1M DoF per rank; replayed as one launch.
   // Captured on a private stream (the caller's may be the null stream), launched on s.
   const auto key = std::make_pair(x_true, y_true);
   auto it = graphs_.find(key);
   if (it == graphs_.end())
   {
      if (graphs_.size() >= kMaxGraphs) { drop_graphs(); }  // callers cycling through temporaries
      if (!cap_) { ECM2_HIP(hipStreamCreateWithFlags(&cap_, hipStreamNonBlocking)); }
      hipGraph_t g = nullptr;
      hipGraphExec_t ge = nullptr;
      ECM2_HIP(hipStreamBeginCapture(cap_, hipStreamCaptureModeThreadLocal));
      try
      {
         mult_stages(x_true, y_true, cap_);
      }
      catch (...)
      {
         (void)hipStreamEndCapture(cap_, &g);  // abandon; every rank fails the same way
         if (g) { (void)hipGraphDestroy(g); }
         (void)hipGetLastError();
         graph_failed_ = true;
         mult_stages(x_true, y_true, s);
         return;
      }
      ECM2_HIP(hipStreamEndCapture(cap_, &g));
      const hipError_t ie = hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
      (void)hipGraphDestroy(g);
      if (ie != hipSuccess)
      {
         (void)hipGetLastError();
         graph_failed_ = true;
         mult_stages(x_true, y_true, s);
         return;
      }
      it = graphs_.emplace(key, ge).first;
   }
   ECM2_HIP(hipGraphLaunch(it->second, s));
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
   diag_local(d_true, s);
   if (part_.overlap) { return; }  // owned entries complete locally
   // P^T of the ghost entries, on s
   ECM2_HIP(hipEventRecord(ev_xg_, s));
   ECM2_HIP(hipStreamWaitEvent(cs_, ev_xg_, 0));
   rccl_exchange(true, nullptr, cs_);
   ECM2_HIP(hipEventRecord(ev_done_, cs_));
   ECM2_HIP(hipStreamWaitEvent(s, ev_done_, 0));
   phase_finish(d_true, s);
}

void ParPAForm::allreduce_sum(double *dev, int n, hipStream_t s)
{
   ECM2_VERIFY(comm_, ERR_STATE, "allreduce needs the RCCL transport");
   ECM2_NCCL(ncclAllReduce(dev, dev, n, ncclFloat64, ncclSum, (ncclComm_t)comm_, s));
}

namespace
{
// The loopback transport of one exchange: every receive of member r copies, on r's comm
// stream and after the peer's `ready` event, the matching send of the peer's schedule (the
// one addressed to r: a pair of ranks exchanges one block per direction).
void group_exchange(std::vector<ParPAForm *> &forms, const std::vector<const double *> &x, bool transpose,
                    hipEvent_t (ParPAForm::*ready)() const)
{
   const int n = (int)forms.size();
   for (int r = 0; r < n; r++)
   {
      ParPAForm &f = *forms[r];
      for (const Xfer &t : f.schedule(transpose))
      {
         if (t.send) { continue; }
         ECM2_VERIFY(t.peer >= 0 && t.peer < n, ERR_INTERNAL, "exchange peer " << t.peer << " outside the group");
         ParPAForm &o = *forms[t.peer];
         const Xfer *m = nullptr;
         for (const Xfer &u : o.schedule(transpose))
         {
            if (u.send && u.peer == r) { m = &u; break; }
         }
         ECM2_VERIFY(m && m->count == t.count, ERR_INTERNAL,
                     "exchange schedules of ranks " << r << " and " << t.peer << " do not match");
         ECM2_HIP(hipStreamWaitEvent(f.comm_stream(), (o.*ready)(), 0));
         ECM2_HIP(hipMemcpyAsync(f.xfer_ptr(t, x[r]), o.xfer_ptr(*m, x[t.peer]), t.count * sizeof(double),
                                 hipMemcpyDeviceToDevice, f.comm_stream()));
      }
   }
}
// The loopback transport of one exchange on one stream (the serial schedule): every receive
// copies the peer's matching send.  comm (a one-rank RCCL communicator): every (send row,
// receive row) pair is instead one ncclSend + ncclRecv of the communicator to itself, all in one
// group -- the rows, buffers and counts of ParPAForm::rccl_exchange through RCCL's own transfer
// path (RCCL matches a group's self sends and receives in issue order).
void group_copies(std::vector<ParPAForm *> &forms, const std::vector<const double *> &x, bool transpose,
                  hipStream_t s, int only = -1, void *comm = nullptr)
{
   const int n = (int)forms.size();
   if (comm) { ECM2_NCCL(ncclGroupStart()); }
   for (int r = 0; r < n; r++)
   {
      if (only >= 0 && r != only) { continue; }
      ParPAForm &f = *forms[r];
      for (const Xfer &t : f.schedule(transpose))
      {
         if (t.send) { continue; }
         ECM2_VERIFY(t.peer >= 0 && t.peer < n, ERR_INTERNAL, "exchange peer " << t.peer << " outside the group");
         ParPAForm &o = *forms[t.peer];
         const Xfer *m = nullptr;
         for (const Xfer &u : o.schedule(transpose))
         {
            if (u.send && u.peer == r) { m = &u; break; }
         }
         ECM2_VERIFY(m && m->count == t.count, ERR_INTERNAL,
                     "exchange schedules of ranks " << r << " and " << t.peer << " do not match");
         double *dst = f.xfer_ptr(t, x.empty() ? nullptr : x[r]);
         const double *src = o.xfer_ptr(*m, x.empty() ? nullptr : x[t.peer]);
         if (comm)
         {
            ECM2_NCCL(ncclSend(src, t.count, ncclFloat64, 0, (ncclComm_t)comm, s));
            ECM2_NCCL(ncclRecv(dst, t.count, ncclFloat64, 0, (ncclComm_t)comm, s));
         }
         else { ECM2_HIP(hipMemcpyAsync(dst, src, t.count * sizeof(double), hipMemcpyDeviceToDevice, s)); }
      }
   }
   if (comm) { ECM2_NCCL(ncclGroupEnd()); }
}

// One-rank communicator of the RCCL-self group transport (created on first use, outside any
// stream capture; lives for the process).
void *self_comm()
{
   static ncclComm_t comm = [] {
      ncclUniqueId id;
      ECM2_NCCL(ncclGetUniqueId(&id));
      ncclComm_t c;
      ECM2_NCCL(ncclCommInitRank(&c, 1, id, 0));
      return c;
   }();
   return comm;
}
} // namespace

void group_self_allreduce(double *dev, int n, hipStream_t s)
{
   ECM2_NCCL(ncclAllReduce(dev, dev, n, ncclFloat64, ncclSum, (ncclComm_t)self_comm(), s));
}

void par_group_mult_member(std::vector<ParPAForm *> &forms, const std::vector<const double *> &x,
                           const std::vector<double *> &y, int r, hipStream_t s)
{
   const int n = (int)forms.size();
   ECM2_VERIFY((int)x.size() == n && (int)y.size() == n, ERR_ARG, "group size mismatch");
   ECM2_VERIFY(r >= 0 && r < n, ERR_ARG, "member " << r << " outside the group of " << n);
   ParPAForm &f = *forms[r];
   ECM2_VERIFY(f.part().rank == r && f.part().nranks == n, ERR_ARG, "loopback group: form " << r << " has rank "
                                                                    << f.part().rank);
   ECM2_VERIFY(f.part().overlap || f.serial(), ERR_UNSUPPORTED,
               "a member's RAP rows alone run the serial schedule");
   ECM2_VERIFY(f.local().assembled(), ERR_STATE, "Mult before Assemble");
   for (const Xfer &t : f.schedule(false))
   {
      if (t.send) { continue; }
      const Xfer *m = nullptr;
      for (const Xfer &u : forms[t.peer]->schedule(false))
      {
         if (u.send && u.peer == r) { m = &u; break; }
      }
      ECM2_VERIFY(m && m->count == t.count, ERR_INTERNAL, "exchange schedules of ranks " << r << " and " << t.peer
                                                                                       << " do not match");
   }
   // the peers' packed sends (and, RAP, their y ghost blocks) are copied as their last group Mult
   // left them: it must have run on these x arrays and on the current assembly
   for (int tr = 0; tr < (f.part().overlap ? 1 : 2); tr++)
   {
      for (const Xfer &t : f.schedule(tr == 1))
      {
         if (t.send) { continue; }
         ParPAForm &o = *forms[t.peer];
         const bool needs = tr == 1 || o.pack_needed();  // P^T: the peer's y ghost block; P: its packed sends
         ECM2_VERIFY(!needs || o.group_mult_current(x[t.peer]), ERR_STATE,
                     "member " << r << ": peer " << t.peer << "'s last group Mult ran on another x or assembly "
                               "(run a group Mult on the same x first)");
      }
   }
   if (f.serial())
   {
      // the rank's own pack (its sends); the peers' packed sends are as their last group Mult left them
      if (f.pack_needed()) { kern::gather_idx((int)f.part().send_idx.size(), f.send_idx_data(), x[r], f.sendbuf_data(), s); }
      group_copies(forms, x, false, s, r);
      f.stage_serial_apply(x[r], y[r], s);  // RAP: + the ghost dofs' sums
      // RAP: the P^T receive copies the peers' ghost contributions -- their y ghost blocks as
      // their own stage_serial_apply left them (a previous group Mult on the same x)
      if (!f.part().overlap) { group_copies(forms, x, true, s, r); }
      f.local().finish_shared(0, f.local().n_shared_owned(), y[r], f.yghost(), s);
      if (!f.part().overlap) { f.phase_finish(y[r], s); }
      return;
   }
   f.stage_pack(x[r], y[r], s);
   // the P exchange of this member on its comm stream: the peers' owned values straight from their x
   for (const Xfer &t : f.schedule(false))
   {
      if (t.send) { continue; }
      ParPAForm &o = *forms[t.peer];
      for (const Xfer &u : o.schedule(false))
      {
         if (u.send && u.peer == r)
         {
            ECM2_HIP(hipMemcpyAsync(f.xfer_ptr(t, x[r]), o.xfer_ptr(u, x[t.peer]), t.count * sizeof(double),
                                    hipMemcpyDeviceToDevice, f.comm_stream()));
            break;
         }
      }
   }
   f.stage_interior(x[r], y[r], s);
   f.stage_boundary(x[r], y[r]);
   f.stage_finish(y[r], s);
}

void par_group_mult(std::vector<ParPAForm *> &forms, const std::vector<const double *> &x,
                    const std::vector<double *> &y, hipStream_t s, bool rccl_self)
{
   const int n = (int)forms.size();
   ECM2_VERIFY((int)x.size() == n && (int)y.size() == n, ERR_ARG, "group size mismatch");
   for (int r = 0; r < n; r++)
   {
      ECM2_VERIFY(forms[r]->part().rank == r && forms[r]->part().nranks == n, ERR_ARG,
                  "loopback group: form " << r << " has rank " << forms[r]->part().rank);
      ECM2_VERIFY(forms[r]->local().assembled(), ERR_STATE, "Mult before Assemble");
   }
   for (int r = 1; r < n; r++)
   {
      ECM2_VERIFY(forms[r]->serial() == forms[0]->serial(), ERR_ARG, "loopback group: members use different schedules");
   }
   ECM2_VERIFY(!rccl_self || forms.empty() || forms[0]->serial(), ERR_UNSUPPORTED,
               "the RCCL-self group transport runs the serial schedule");
   void *comm = rccl_self ? self_comm() : nullptr;
   for (int r = 0; r < n; r++) { forms[r]->note_group_mult(x[r]); }
   if (!forms.empty() && forms[0]->serial())
   {
      // the serial schedule, stage-major on s: packs, the P copies, the applies, [RAP: P^T
      // copies], the sums
      for (int r = 0; r < n; r++)
      {
         ParPAForm &f = *forms[r];
         if (f.pack_needed())
         {
            kern::gather_idx((int)f.part().send_idx.size(), f.send_idx_data(), x[r], f.sendbuf_data(), s);
         }
      }
      group_copies(forms, x, false, s, -1, comm);
      for (int r = 0; r < n; r++) { forms[r]->stage_serial_apply(x[r], y[r], s); }
      if (!forms[0]->part().overlap) { group_copies(forms, x, true, s, -1, comm); }
      for (int r = 0; r < n; r++)
      {
         forms[r]->local().finish_shared(0, forms[r]->local().n_shared_owned(), y[r], forms[r]->yghost(), s);
         if (!forms[r]->part().overlap) { forms[r]->phase_finish(y[r], s); }
      }
      return;
   }
   // the same stages as ParPAForm::mult, stage-major over the members; a member's
   // exchanges wait for its peers' events and copy from their buffers on its comm stream
   for (int r = 0; r < n; r++) { forms[r]->stage_pack(x[r], y[r], s); }
   group_exchange(forms, x, false, &ParPAForm::event_packed);
   for (int r = 0; r < n; r++) { forms[r]->stage_boundary(x[r], y[r]); }
   if (!forms.empty() && !forms[0]->part().overlap) { group_exchange(forms, x, true, &ParPAForm::event_ghosts_summed); }
   for (int r = 0; r < n; r++) { forms[r]->stage_interior(x[r], y[r], s); }
   for (int r = 0; r < n; r++) { forms[r]->stage_finish(y[r], s); }
}

void par_group_diagonal(std::vector<ParPAForm *> &forms, const std::vector<double *> &d, hipStream_t s)
{
   ECM2_VERIFY(d.size() == forms.size(), ERR_ARG, "group size mismatch");
   for (size_t r = 0; r < forms.size(); r++) { forms[r]->diag_local(d[r], s); }
   if (forms.empty() || forms[0]->part().overlap) { return; }  // owned entries complete locally
   // P^T of the ghost entries: everything on s (the comm streams wait for it)
   hipEvent_t ev;
   ECM2_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
   ECM2_HIP(hipEventRecord(ev, s));
   for (ParPAForm *f : forms) { ECM2_HIP(hipStreamWaitEvent(f->comm_stream(), ev, 0)); }
   std::vector<const double *> none(forms.size(), nullptr);
   for (ParPAForm *f : forms) { ECM2_HIP(hipEventRecord(f->event_ghosts_summed(), f->comm_stream())); }
   group_exchange(forms, none, true, &ParPAForm::event_ghosts_summed);
   for (ParPAForm *f : forms)
   {
      ECM2_HIP(hipEventRecord(ev, f->comm_stream()));
      ECM2_HIP(hipStreamWaitEvent(s, ev, 0));
   }
   (void)hipEventDestroy(ev);
   for (size_t r = 0; r < forms.size(); r++) { forms[r]->phase_finish(d[r], s); }
}

} // namespace ecm2
