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
      ECM2_HIP(hipMemcpy(a.data(), h.data(), sizeof(double) * n, hipMemcpyHostToDevice));
      ECM2_HIP(hipMemset(b.data(), 0, sizeof(double) * n));
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
      ECM2_HIP(hipMemcpy(r.data(), b.data(), sizeof(double) * n, hipMemcpyDeviceToHost));
      for (int i = 0; i < n; i++) { err = std::max(err, std::fabs(r[i] - h[i])); }
      if (graph && rep == 2) { ECM2_HIP(hipGraphExecDestroy(ge)); ge = nullptr; }
   }
   ECM2_HIP(hipStreamDestroy(st));
   (void)ncclCommDestroy(comm);
   return err;
}

// CUs reserved for the comm stream (RCCL kernels, boundary elements, ghost sums): the
// interior kernel runs on a stream masked to the other CUs, so the exchange chain never
// waits for the interior's waves to retire (at C2 size one interior wave lives for the
// whole kernel).  ECM2_COMM_CUS=0: no masks (comm stream by priority only).
static int comm_cus()
{
   static const int v = [] {
      const char *e = std::getenv("ECM2_COMM_CUS");
      return e ? std::max(0, std::atoi(e)) : 0;
   }();
   return v;
}

// Interior split (percent of the interior blocks in part A, 0 = none): part A runs while the
// exchange and the boundary elements proceed on the comm stream, part B waits for the
// boundary kernel -- so the boundary never queues behind a full-GPU interior kernel whose
// waves all live for the kernel's whole duration.  ECM2_INTERIOR_SPLIT.
static int interior_split_pct()
{
   static const int v = [] {
      const char *e = std::getenv("ECM2_INTERIOR_SPLIT");
      return e ? std::max(0, std::min(100, std::atoi(e))) : 0;
   }();
   return v;
}

// Boundary elements with the plane-per-wave latency kernel (ECM2_BOUNDARY_PP=0: the
// throughput kernel, whose waves each walk all planes).
static bool boundary_pp()
{
   static const bool v = [] {
      const char *e = std::getenv("ECM2_BOUNDARY_PP");
      return !(e && std::string(e) == "0");
   }();
   return v;
}

// ECM2_PAR_GRAPH=0: launch the Mult's stages directly instead of replaying a captured graph.
static bool par_graph()
{
   static const bool v = [] {
      const char *e = std::getenv("ECM2_PAR_GRAPH");
      return !(e && std::string(e) == "0");
   }();
   return v;
}

ParPAForm::ParPAForm(const LocalPart &part, const double *enodes_local_host, int q1d,
                     const unsigned char *rccl_id)
   : part_(part)
{
   const int nl = part.n_owned + part.n_ghost;
   local_.reset(new PAForm(part.ne_local, part.order, nl, part.gather_map.data(), q1d, part.n_owned));
   local_->set_element_nodes(enodes_local_host);
   // the Mult applies blocks [0, b_split) and [b_split, b_int) (interior parts A, B) and
   // [b_int, nblk) (boundary) separately
   const int bi = part.ne_interior / kElemBlock;
   b_split_ = (int)((long)bi * interior_split_pct() / 100);
   if (b_split_ <= 0 || b_split_ >= bi) { b_split_ = 0; }
   if (b_split_) { local_->set_block_splits({b_split_, bi}); }
   else { local_->set_block_splits({bi}); }
   if (boundary_pp()) { local_->set_latency_from(bi); }  // boundary blocks: one block per workgroup
   send_idx_.upload(part.send_idx);
   pack_needed_ = false;
   for (size_t k = 0; k < part.nbrs.size(); k++)
   {
      const int i0 = part.send_off[k], i1 = part.send_off[k + 1];
      bool contig = i1 > i0;
      for (int i = i0 + 1; i < i1 && contig; i++) { contig = part.send_idx[i] == part.send_idx[i - 1] + 1; }
      send_start_.push_back(contig ? part.send_idx[i0] : -1);
      pack_needed_ |= !contig && i1 > i0;
   }
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
   int dev = 0, ncu = 0;
   ECM2_HIP(hipGetDevice(&dev));
   ECM2_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
   const int k = comm_cus();
   if (k > 0 && 4 * k <= ncu)
   {
      // k / 8 CUs of every 32 (one XCD's worth): balanced over the XCDs whether the mask is
      // read linearly or per XCD
      const int per = std::max(1, k / 8);
      std::vector<uint32_t> cm((ncu + 31) / 32, 0u), im((ncu + 31) / 32, 0u);
      for (int i = 0; i < ncu; i++) { (i % 32 < per ? cm : im)[i / 32] |= 1u << (i % 32); }
      ECM2_HIP(hipExtStreamCreateWithCUMask(&cs_, (uint32_t)cm.size(), cm.data()));
      ECM2_HIP(hipExtStreamCreateWithCUMask(&is_, (uint32_t)im.size(), im.data()));
      ECM2_HIP(hipEventCreateWithFlags(&ev_s_, hipEventDisableTiming));
      ECM2_HIP(hipEventCreateWithFlags(&ev_int_, hipEventDisableTiming));
   }
   else
   {
      int prio_least = 0, prio_greatest = 0;
      ECM2_HIP(hipDeviceGetStreamPriorityRange(&prio_least, &prio_greatest));
      ECM2_HIP(hipStreamCreateWithPriority(&cs_, hipStreamNonBlocking, prio_greatest));
   }
   ECM2_HIP(hipEventCreateWithFlags(&ev_pack_, hipEventDisableTiming));
   ECM2_HIP(hipEventCreateWithFlags(&ev_xg_, hipEventDisableTiming));
   ECM2_HIP(hipEventCreateWithFlags(&ev_yg_, hipEventDisableTiming));
   ECM2_HIP(hipEventCreateWithFlags(&ev_done_, hipEventDisableTiming));
   ECM2_HIP(hipEventCreateWithFlags(&ev_bnd_, hipEventDisableTiming));
   ECM2_HIP(hipDeviceSynchronize());
}

ParPAForm::~ParPAForm()
{
   if (comm_) { (void)ncclCommDestroy((ncclComm_t)comm_); }
   if (cs_) { (void)hipStreamDestroy(cs_); }
   if (is_) { (void)hipStreamDestroy(is_); }
   for (auto &kv : graphs_) { (void)hipGraphExecDestroy(kv.second); }
   if (cap_) { (void)hipStreamDestroy(cap_); }
   for (hipEvent_t e : {ev_pack_, ev_xg_, ev_yg_, ev_done_, ev_s_, ev_int_, ev_bnd_})
   {
      if (e) { (void)hipEventDestroy(e); }
   }
}

void ParPAForm::assemble(hipStream_t s) { local_->assemble(s); }

size_t ParPAForm::algorithmic_bytes() const
{
   // SURVEY §8(d) over the rank's own elements and true dofs (OVERLAP's ghost elements are
   // duplicated work, not counted)
   const PAForm &f = *local_;
   const size_t nq = (size_t)f.q1d() * f.q1d() * f.q1d(), nd = (size_t)f.d1d() * f.d1d() * f.d1d();
   const size_t nc = (f.has_diffusion() ? 6 : 0) + (f.has_mass() ? 1 : 0);
   return 8ull * part_.ne_owned * nq * nc + 16ull * part_.n_owned + 4ull * part_.ne_owned * nd;
}

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
   const int b_int = part_.ne_interior / kElemBlock;
   local_->record_start_public(cs_);
   local_->apply_blocks(x_true, xg_.data(), y_true, yg_.data(), b_int, local_->nblocks(), cs_, boundary_pp());
   local_->record_stop_public(cs_);
   ECM2_HIP(hipEventRecord(ev_bnd_, cs_));
   // ghost dofs are touched only by boundary elements: their sums are complete here (OVERLAP:
   // the ghost outputs are discarded, nothing to sum)
   if (!part_.overlap) { local_->finish_shared(local_->n_shared_owned(), local_->n_shared(), y_true, yg_.data(), cs_); }
   ECM2_HIP(hipEventRecord(ev_yg_, cs_));
}

void ParPAForm::stage_interior(const double *x_true, double *y_true, hipStream_t s)
{
   const int b_int = part_.ne_interior / kElemBlock;
   hipStream_t st = s;
   if (is_)  // interior on the CU-masked stream, ordered after s's work so far
   {
      ECM2_HIP(hipEventRecord(ev_s_, s));
      ECM2_HIP(hipStreamWaitEvent(is_, ev_s_, 0));
      st = is_;
   }
   if (b_split_)
   {
      local_->record_start_public(st);
      local_->apply_blocks(x_true, xg_.data(), y_true, yg_.data(), 0, b_split_, st);
      local_->record_stop_public(st);
      ECM2_HIP(hipStreamWaitEvent(st, ev_bnd_, 0));
      local_->record_start_public(st);
      local_->apply_blocks(x_true, xg_.data(), y_true, yg_.data(), b_split_, b_int, st);
      local_->record_stop_public(st);
   }
   else
   {
      local_->record_start_public(st);
      local_->apply_blocks(x_true, xg_.data(), y_true, yg_.data(), 0, b_int, st);
      local_->record_stop_public(st);
   }
   if (is_)
   {
      ECM2_HIP(hipEventRecord(ev_int_, is_));
      ECM2_HIP(hipStreamWaitEvent(s, ev_int_, 0));
   }
}

void ParPAForm::stage_finish(double *y_true, hipStream_t s)
{
   ECM2_HIP(hipEventRecord(ev_done_, cs_));
   if (part_.overlap)
   {
      // every contribution to an owned dof was computed here: sum the shared ones, done
      ECM2_HIP(hipStreamWaitEvent(s, ev_done_, 0));
      local_->finish_shared(0, local_->n_shared_owned(), y_true, yg_.data(), s);
      return;
   }
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
         if (nown) { ECM2_NCCL(ncclSend(send_ptr(k, x_cur_), nown, ncclFloat64, part_.nbrs[k], comm, cs_)); }
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

// Measurement aid (ECM2_EMULATE_EXCHANGE=1, no RCCL communicator): one rank of an N-rank
// partition run alone on one GPU, each exchange replaced by same-size device copies from the
// rank's own buffers on the comm stream.  The values are NOT the operator's; the stream /
// event / CU structure and every kernel are the RCCL rank's, so its timeline shows whether
// the boundary chain hides behind the interior (bench.py --emulate-rank).
static bool emulate_exchange()
{
   static const bool v = [] {
      const char *e = std::getenv("ECM2_EMULATE_EXCHANGE");
      return e && std::string(e) == "1";
   }();
   return v;
}

void ParPAForm::self_exchange(bool transpose)
{
   for (size_t k = 0; k < part_.nbrs.size(); k++)
   {
      const size_t nown = part_.send_off[k + 1] - part_.send_off[k];
      const size_t ngh = part_.recv_off[k + 1] - part_.recv_off[k];
      if (!transpose && ngh)
      {
         // a same-size copy from this rank's own send range stands in for the peer's
         const size_t n = std::min(ngh, nown ? nown : sendbuf_.size());
         const double *src = nown ? send_ptr((int)k, x_cur_) : sendbuf_.data();
         ECM2_HIP(hipMemcpyAsync(xg_.data() + part_.recv_off[k], src, n * sizeof(double),
                                 hipMemcpyDeviceToDevice, cs_));
      }
      if (transpose && nown)
      {
         const size_t n = std::min(nown, yg_.size());
         ECM2_HIP(hipMemcpyAsync(rbuf_.data() + part_.send_off[k], yg_.data(), n * sizeof(double),
                                 hipMemcpyDeviceToDevice, cs_));
      }
   }
}

// Enqueue the interior elements before the exchange chain (ECM2_INTERIOR_FIRST=0: after):
// each host call costs microseconds, so whatever is enqueued first starts first; the
// interior kernel leaves wave slots free for the comm stream's boundary kernel.
static bool interior_first()
{
   static const bool v = [] {
      const char *e = std::getenv("ECM2_INTERIOR_FIRST");
      return !(e && std::string(e) == "0");
   }();
   return v;
}

// OVERLAP with the boundary on the caller's stream after the interior (ECM2_PAR_SERIAL=1):
// only the exchange runs on the comm stream, and the one cross-stream wait (for P) is long
// satisfied when the interior ends -- no join after the boundary kernel.
static bool par_serial()
{
   static const bool v = [] {
      const char *e = std::getenv("ECM2_PAR_SERIAL");
      return e && std::string(e) == "1";
   }();
   return v;
}

void ParPAForm::mult_stages(const double *x_true, double *y_true, hipStream_t s, bool emu)
{
   x_cur_ = x_true;
   if (part_.overlap && par_serial() && !b_split_ && !is_)
   {
      stage_pack(x_true, y_true, s);
      stage_interior(x_true, y_true, s);
      if (emu) { self_exchange(false); } else { rccl_exchange(false); }
      ECM2_HIP(hipEventRecord(ev_done_, cs_));
      ECM2_HIP(hipStreamWaitEvent(s, ev_done_, 0));
      local_->record_start_public(s);
      local_->apply_blocks(x_true, xg_.data(), y_true, yg_.data(), b_int(), local_->nblocks(), s, boundary_pp());
      local_->record_stop_public(s);
      local_->finish_shared(0, local_->n_shared_owned(), y_true, yg_.data(), s);
      return;
   }
   const bool first = interior_first() && !b_split_;  // part B of a split waits for the boundary
   stage_pack(x_true, y_true, s);
   if (first) { stage_interior(x_true, y_true, s); }
   if (emu) { self_exchange(false); } else { rccl_exchange(false); }
   stage_boundary(x_true, y_true);
   if (!part_.overlap)
   {
      if (emu) { self_exchange(true); } else { rccl_exchange(true); }
   }
   if (!first) { stage_interior(x_true, y_true, s); }
   stage_finish(y_true, s);
}

void ParPAForm::mult(const double *x_true, double *y_true, hipStream_t s)
{
   const bool emu = !comm_ && emulate_exchange();
   ECM2_VERIFY(comm_ || emu, ERR_STATE, "mult needs the RCCL transport (use the loopback group otherwise)");
   if (!par_graph() || graph_failed_ || local_->timing_on() || !p2p_warm_)
   {
      // the first Mult runs directly on every rank: RCCL sets up its peer connections
      // lazily at the first send/recv, which then happens outside a stream capture
      mult_stages(x_true, y_true, s, emu);
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
      if (!cap_) { ECM2_HIP(hipStreamCreateWithFlags(&cap_, hipStreamNonBlocking)); }
      hipGraph_t g = nullptr;
      hipGraphExec_t ge = nullptr;
      ECM2_HIP(hipStreamBeginCapture(cap_, hipStreamCaptureModeThreadLocal));
      try
      {
         mult_stages(x_true, y_true, cap_, emu);
      }
      catch (...)
      {
         (void)hipStreamEndCapture(cap_, &g);  // abandon; every rank fails the same way
         if (g) { (void)hipGraphDestroy(g); }
         (void)hipGetLastError();
         graph_failed_ = true;
         mult_stages(x_true, y_true, s, emu);
         return;
      }
      ECM2_HIP(hipStreamEndCapture(cap_, &g));
      const hipError_t ie = hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
      (void)hipGraphDestroy(g);
      if (ie != hipSuccess)
      {
         (void)hipGetLastError();
         graph_failed_ = true;
         mult_stages(x_true, y_true, s, emu);
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
   ncclComm_t comm = (ncclComm_t)comm_;
   diag_local(d_true, s);
   if (part_.overlap) { return; }  // owned entries complete locally
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
         ECM2_HIP(hipMemcpyAsync(f.xghost() + pr.recv_off[k], forms[o]->send_ptr(j, x[o]),
                                 cnt * sizeof(double), hipMemcpyDeviceToDevice, f.comm_stream()));
      }
   }
   for (int r = 0; r < n; r++) { forms[r]->stage_boundary(x[r], y[r]); }
   for (int r = 0; r < n; r++)
   {
      ParPAForm &f = *forms[r];
      if (f.part().overlap) { continue; }  // no P^T
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
   if (!forms.empty() && forms[0]->part().overlap) { return; }  // owned entries complete locally
   group_reduce_ghosts(forms, d, s);
}
} // namespace ecm2
