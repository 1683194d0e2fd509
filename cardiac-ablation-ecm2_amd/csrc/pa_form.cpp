// pa_form.cpp -- see pa_form.hpp.
#include "pa_form.hpp"
#include "bricks.hpp"

#include <algorithm>
#include <climits>
#include <map>
#include <tuple>
#include <array>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <string>
#include <unordered_map>

namespace ecm2
{

void require_device()
{
   int n = 0;
   const hipError_t e = hipGetDeviceCount(&n);
   ECM2_VERIFY(e == hipSuccess && n > 0, ERR_HIP,
               "no HIP device available (the PA path has no CPU fallback)");
}

PAForm::PAForm(int ne, int order, int ndofs, const int *gather_map_host, int q1d, int n_owned)
   : ne_(ne), order_(order), ndofs_(ndofs), n_owned_(n_owned < 0 ? ndofs : n_owned)
{
   ECM2_VERIFY(n_owned_ <= ndofs, ERR_ARG, "n_owned > ndofs");
   ECM2_VERIFY(ne >= 0 && ndofs >= 0, ERR_ARG, "negative sizes");
   ECM2_VERIFY(order >= 1 && order + 1 <= MAX_D1D, ERR_ARG, "unsupported order " << order);
   ECM2_VERIFY(ne == 0 || gather_map_host != nullptr, ERR_ARG, "null gather map");
   require_device();
   D_ = order + 1;
   Q_ = q1d > 0 ? q1d : default_q1d(order);
   ECM2_VERIFY(Q_ >= D_ && Q_ <= MAX_Q1D, ERR_ARG, "q1d must satisfy p+1 <= q1d <= " << MAX_Q1D);
   ND_ = D_ * D_ * D_;
   NQ_ = Q_ * Q_ * Q_;
   maps_ = make_dof_to_quad(order, Q_);
   basis_ = make_basis1d(maps_);
   basis1_ = make_basis1d(make_dof_to_quad(1, Q_));
   gmap_host_.assign(gather_map_host, gather_map_host + (size_t)ne * ND_);
   for (int g : gmap_host_)
   {
      const int d = g >= 0 ? g : -1 - g;
      ECM2_VERIFY(d >= 0 && d < ndofs, ERR_ARG, "gather map entry " << g << " out of range [0," << ndofs << ")");
   }
   gmap_.upload(gmap_host_);
   W_.upload(maps_.W);
   layout_.ne = ne;
   layout_.nq = NQ_;
}

PAForm::~PAForm()
{
   for (auto &e : ev_start_) { (void)hipEventDestroy(e); }
   for (auto &e : ev_stop_) { (void)hipEventDestroy(e); }
}

// Every element a parallelepiped: the trilinear map's bilinear and trilinear terms vanish
// (to 1e-13 of the element's edge length, i.e. below the operator's 1e-12 parity bar), so
// its Jacobian is constant.  Terms are differences of edge vectors (exact for lattices).
static bool all_affine(int ne, const double *X)
{
   for (int e = 0; e < ne; e++)
   {
      const double *p = X + (size_t)e * 24;
      double h = 0.0, dev = 0.0;
      for (int i = 0; i < 3; i++)
      {
         const double *c = p + i * 8;  // corner a = ax + 2 ay + 4 az
         const double ex = c[1] - c[0], ey = c[2] - c[0], ez = c[4] - c[0];
         h = std::max({h, std::fabs(ex), std::fabs(ey), std::fabs(ez)});
         dev = std::max({dev, std::fabs((c[3] - c[2]) - ex), std::fabs((c[5] - c[4]) - ex),
                         std::fabs((c[6] - c[4]) - ey), std::fabs((c[7] - c[6]) - ex),
                         std::fabs((c[7] - c[5]) - ey), std::fabs((c[7] - c[3]) - ez)});
      }
      if (!(dev <= 1e-13 * h)) { return false; }
   }
   return true;
}

void PAForm::set_element_nodes(const double *enodes_host)
{
   ECM2_VERIFY(ne_ == 0 || enodes_host, ERR_ARG, "null element nodes");
   enodes_.upload(enodes_host, (size_t)ne_ * 24);
   ECM2_HIP(hipDeviceSynchronize());
   affine_ = all_affine(ne_, enodes_host);
   jac_ = nullptr;
   assembled_ = false;
}

void PAForm::set_jacobians(const double *J_device)
{
   ECM2_VERIFY(ne_ == 0 || J_device, ERR_ARG, "null Jacobian array");
   jac_ = J_device;
   affine_ = false;
   assembled_ = false;
}

void PAForm::set_geometry_compression(bool on)
{
   compress_ = on;
   assembled_ = false;
}

void PAForm::set_coefficient_snapshot(bool on)
{
   tsnap_pref_ = on;
   assembled_ = false;
}

void PAForm::set_block_splits(const std::vector<int> &splits)
{
   for (int b : splits) { ECM2_VERIFY(b >= 0 && b <= layout_.nblk(), ERR_ARG, "block split " << b << " out of range"); }
   splits_ = splits;
   gmap_line_.resize(0);
   if (perm_auto_)  // the derived brick order respects the segments: derive it again
   {
      perm_host_.clear();
      perm_auto_ = false;
      gmap_blk_.resize(0);
   }
   assembled_ = false;
}

void PAForm::set_latency_from(int b)
{
   latency_from_ = b;
   gmap_blk_.resize(0);  // the face-assembly plan depends on it: rebuild
   assembled_ = false;
}

void PAForm::set_line_bricks(int bz)
{
   ECM2_VERIFY(bz >= -1 && bz <= 2, ERR_ARG, "brick mode " << bz << " not in {-1, 0, 1, 2}");
   line_bricks_ = bz;
   gmap_line_.resize(0);
   assembled_ = false;
}

void PAForm::set_attributes(const int *attr_host)
{
   ECM2_VERIFY(ne_ == 0 || attr_host, ERR_ARG, "null attribute array");
   attr_.assign(attr_host, attr_host + ne_);
   assembled_ = false;
}

void PAForm::add_integrator(int kind, const CoeffDesc &c, const int *marker, int n_marker)
{
   ECM2_VERIFY(!marker || n_marker >= 0, ERR_ARG, "negative marker size");
   ECM2_VERIFY(kind == INTEG_MASS || kind == INTEG_DIFFUSION, ERR_ARG, "unknown integrator " << kind);
   ECM2_VERIFY(c.kind >= COEFF_CONSTANT && c.kind <= COEFF_GRIDFUNC, ERR_ARG, "unknown coefficient kind " << c.kind);
   ECM2_VERIFY(c.dim() == 1 || kind == INTEG_DIFFUSION, ERR_ARG,
               "vector / matrix coefficients belong to a DiffusionIntegrator");
   ECM2_VERIFY(!c.quad_values() || ne_ == 0 || c.quad, ERR_ARG, "null quadrature coefficient");
   ECM2_VERIFY(!c.gridfunc() || ndofs_ == 0 || c.lvec, ERR_ARG, "null grid function");
   if (kind == INTEG_MASS)
   {
      ECM2_VERIFY(!have_mass_, ERR_UNSUPPORTED, "a MassIntegrator is already present");
      have_mass_ = true;
      cmass_ = c;
   }
   else
   {
      ECM2_VERIFY(!have_diff_, ERR_UNSUPPORTED, "a DiffusionIntegrator is already present");
      have_diff_ = true;
      cdiff_ = c;
   }
   // (the marker state changes only once the integrator is accepted: a rejected duplicate leaves
   // the installed one untouched)
   marked_[kind] = marker != nullptr;
   marker_[kind].assign(marker, marker ? marker + n_marker : marker);
   order_added_.push_back(kind);
   assembled_ = false;
}

void PAForm::set_element_order(const int *perm)
{
   std::vector<int> seen(ne_, 0);
   perm_host_.assign(perm, perm + ne_);
   perm_auto_ = false;
   for (int e : perm_host_)
   {
      ECM2_VERIFY(e >= 0 && e < ne_ && !seen[e], ERR_ARG, "element order is not a permutation");
      seen[e] = 1;
   }
   gmap_blk_.resize(0);
   gmap_line_.resize(0);
   assembled_ = false;
}

namespace
{
// In-wave face assembly plan for the blocked (64 elements per wave) layout.
// Directions x, y, z pair lane l with l+1, l+4, l+16: lane l adds the partner's
// low face (index 0 along the direction) into its high face (index D-1) when all
// face dofs coincide and no nonzero value could land in an entry that no longer
// holds its dof; the partner then zeroes that face.  After the three passes the
// "holding" entries (holds[(b*64+l)*ND+a]) carry each dof's in-wave sum, and
// hcount[d] counts the holders of dof d in the whole mesh: a dof held once is
// plain-stored, otherwise it is "shared" (partial slot or atomic add).
// In-wave face assembly plan of the blocked layout (see tpe_assemble_store): per 64-lane
// block and direction, lane l receives lane l + off's low face into its high face when the
// faces coincide; then (xwave) across the waves of a workgroup group: a wave whose 16
// high-face lanes all coincide with another wave's 16 low-face lanes receives those through
// LDS.  groups: [first block, end block, link allowed] of every workgroup (<= 4 blocks, in
// the launch's grouping: from each apply segment's first block).  Lane flags: bits 1|4|16 receive x|y|z in-wave, 2|8|32 low face
// sent (in-wave or across waves), 64|128|256 receive x|y|z across waves, bits 9-11 | 12-14 |
// 15-17 the sending wave (within the group) for x | y | z.
void build_merge_plan(int ne, int D, const std::vector<int> &gmap_int, int ndofs,
                      std::vector<char> &holds, std::vector<int> &hcount, std::vector<int> &flags,
                      const std::vector<std::array<int, 3>> &groups)
{
   const int ND = D * D * D, nblk = (ne + 63) / 64;
   flags.assign((size_t)nblk * 64, 0);
   holds.assign((size_t)nblk * 64 * ND, 0);
   hcount.assign(ndofs, 0);
   auto dofv = [](int g) { return g >= 0 ? g : -1 - g; };
   auto face = [D](int dir, int s, int i, int j) {
      if (dir == 0) { return (j * D + i) * D + s; }
      if (dir == 1) { return (j * D + s) * D + i; }
      return (s * D + j) * D + i;
   };
   const int off[3] = {1, 4, 16}, recv[3] = {1, 4, 16}, sent[3] = {2, 8, 32};
   auto act = [&](int b, int l) { return b * 64 + l < ne; };
   auto dof = [&](int b, int l, int a) { return dofv(gmap_int[((size_t)b * 64 + l) * ND + a]); };
   auto H = [&](int b, int l, int a) -> char & { return holds[((size_t)b * 64 + l) * ND + a]; };
   auto F = [&](int b, int l) -> int & { return flags[(size_t)b * 64 + l]; };
   for (int b = 0; b < nblk; b++)
      for (int l = 0; l < 64; l++)
         for (int a = 0; a < ND; a++) { H(b, l, a) = act(b, l); }
   for (const auto &grp : groups)
   {
      const int g0 = grp[0], g1 = grp[1];
      const bool xw = grp[2] != 0;
      for (int dir = 0; dir < 3; dir++)
      {
         for (int b = g0; b < g1; b++)
         {
            for (int l = 0; l + off[dir] < 64; l++)
            {
               const int m = l + off[dir];
               if (!act(b, l) || !act(b, m)) { continue; }
               bool ok = true;
               for (int j = 0; j < D && ok; j++)
                  for (int i = 0; i < D && ok; i++)
                  {
                     const int ar = face(dir, D - 1, i, j), as = face(dir, 0, i, j);
                     ok = dof(b, l, ar) == dof(b, m, as) && (H(b, l, ar) || !H(b, m, as));
                  }
               if (!ok) { continue; }
               F(b, l) |= recv[dir];
               F(b, m) |= sent[dir];
            }
            for (int m = 0; m < 64; m++)
            {
               if (!(F(b, m) & sent[dir])) { continue; }
               for (int j = 0; j < D; j++)
                  for (int i = 0; i < D; i++) { H(b, m, face(dir, 0, i, j)) = 0; }
            }
         }
         if (!xw) { continue; }
         // across the group's waves: wave br's 16 high-face lanes <- wave bs's low-face lanes
         for (int br = g0; br < g1; br++)
         {
            for (int bs = g0; bs < g1; bs++)
            {
               if (bs == br) { continue; }
               bool ok = true;
               for (int l = 0; l < 64 && ok; l++)
               {
                  if ((l / off[dir]) % 4 != 3) { continue; }
                  const int m = l - 3 * off[dir];
                  ok = act(br, l) && act(bs, m) && !(F(bs, m) & sent[dir]);
                  for (int j = 0; j < D && ok; j++)
                     for (int i = 0; i < D && ok; i++)
                     {
                        const int ar = face(dir, D - 1, i, j), as = face(dir, 0, i, j);
                        ok = dof(br, l, ar) == dof(bs, m, as) && H(br, l, ar) && H(bs, m, as);
                     }
               }
               if (!ok) { continue; }
               for (int l = 0; l < 64; l++)
               {
                  if ((l / off[dir]) % 4 != 3) { continue; }
                  const int m = l - 3 * off[dir];
                  F(br, l) |= (64 << dir) | ((bs - g0) << (9 + 3 * dir));
                  F(bs, m) |= sent[dir];
                  for (int j = 0; j < D; j++)
                     for (int i = 0; i < D; i++) { H(bs, m, face(dir, 0, i, j)) = 0; }
               }
               break;  // one sender per receiving wave and direction
            }
         }
      }
   }
   for (int b = 0; b < nblk; b++)
      for (int l = 0; l < 64; l++)
         for (int a = 0; a < ND; a++) { if (H(b, l, a)) { hcount[dof(b, l, a)]++; } }
}
} // namespace

// Second-pass plan of the deterministic scatter: every dof not held exactly once with its
// partial slots in ascending order; dofs held by nobody get an empty list (y = 0).  The
// owned dofs come first, then the ghosts (split form); within each range the list is
// ordered by first slot, so neighbouring threads of k_sum_partials read neighbouring slots.
void PAForm::build_shared_plan(const std::vector<int> &hcount, const std::vector<int> &hdof,
                               const std::vector<int> &hslot, hipStream_t s)
{
   std::vector<int> start(ndofs_ + 1, 0);
   for (int d = 0; d < ndofs_; d++) { start[d + 1] = start[d] + (hcount[d] > 1 ? hcount[d] : 0); }
   ECM2_VERIFY((size_t)start[ndofs_] == hdof.size(), ERR_INTERNAL, "shared holder count mismatch");
   std::vector<int> slots_by_dof(hdof.size()), fill(start.begin(), start.end() - 1);
   for (size_t i = 0; i < hdof.size(); i++) { slots_by_dof[fill[hdof[i]]++] = hslot[i]; }
   std::vector<int> dofs;
   for (int d = 0; d < ndofs_; d++) { if (hcount[d] != 1) { dofs.push_back(d); } }
   auto key = [&](int d) -> long {
      const long first = hcount[d] > 1 ? slots_by_dof[start[d]] : -1;
      return (d < n_owned_ ? 0 : (1l << 40)) + first;
   };
   std::stable_sort(dofs.begin(), dofs.end(), [&](int p, int q) { return key(p) < key(q); });
   ECM2_VERIFY(slots_by_dof.size() < (1ull << 31), ERR_UNSUPPORTED, "too many partial slots");
   n_sh_ = (int)dofs.size();
   n_sh_owned_ = 0;
   while (n_sh_owned_ < n_sh_ && dofs[n_sh_owned_] < n_owned_) { n_sh_owned_++; }
   n_slots_ = (long)slots_by_dof.size();

   // Run compression, per range ([owned | ghost]: finish_shared runs each on its own).  1D runs:
   // consecutive entries (in the order above) with equal holder counts whose dof and every
   // holder's slot advance by the same steps; 2D runs: 1D runs of one shape whose first entries
   // advance by common steps again (a face interior, a 4 x 4 lane patch).  Entries are
   // re-emitted run by run; each dof keeps its holders in ascending slot order.
   auto cnt = [&](int d) { return hcount[d] > 1 ? start[d + 1] - start[d] : 0; };
   auto slot = [&](int d, int h) { return slots_by_dof[start[d] + h]; };
   // d1 == kExplicitDofs: the run's slots are affine but its dofs are not (a numbering that is not a
   // lattice, e.g. the reference's entity numbering): the pass reads each entry's dof from the
   // plan's entry list instead (4 coalesced bytes per entry)
   constexpr int kExplicitDofs = INT32_MIN;
   struct Run { int n1, n2, c, dof0, d1, d2, t1, t2, first; std::vector<int> s0; };
   std::vector<Run> runs;
   std::vector<int> order;  // plan entries (dofs) in run-major order
   for (int range = 0; range < 2; range++)
   {
      const int r0 = range ? n_sh_owned_ : 0, r1 = range ? n_sh_ : n_sh_owned_;
      struct R1 { int i0, n, c, d1, t1; };
      std::vector<R1> r1s;
      // longest run from entry i: slots affine with a common step, dofs too unless explicit
      auto extend = [&](int i, bool explicit_dofs, int &d1, int &t1) {
         const int c = cnt(dofs[i]);
         int n = 1;
         d1 = 0;
         t1 = 0;
         while (i + n < r1 && n < 64 && c <= 8)
         {
            const int dj = dofs[i + n], dp = dofs[i + n - 1];
            if (cnt(dj) != c) { break; }
            const int dd = dj - dp, tt = c ? slot(dj, 0) - slot(dp, 0) : 0;
            bool ok = n == 1 || ((explicit_dofs || dd == d1) && tt == t1);
            for (int h = 1; h < c && ok; h++) { ok = slot(dj, h) - slot(dp, h) == tt; }
            if (!ok) { break; }
            if (n == 1) { d1 = dd; t1 = tt; }
            n++;
         }
         return n;
      };
      for (int i = r0; i < r1;)
      {
         const int c = cnt(dofs[i]);
         int d1, t1, e1, et1;
         int n = extend(i, false, d1, t1);
         const int n_ex = c ? extend(i, true, e1, et1) : 0;  // explicit-dof run length
         if (n_ex > n && (n < 4 || n_ex >= 2 * n))  // a short affine run costs more descriptor bytes per entry
         {
            n = n_ex;
            d1 = kExplicitDofs;
            t1 = et1;
         }
         r1s.push_back({i, n, c, d1, t1});
         i += n;
      }
      // 2D: one open run per (count, length, steps) class; a 1D run joins its class's open run
      // when its first entry continues that run's lattice, else it opens a new one.  A run whose
      // slots continue the lattice but whose dofs do not (the reference's numbering: the 3- and
      // 4-holder entries of a brick edge are 1D runs of one entry each) joins the last open run
      // of its (count, length, slot step) class instead, which becomes explicit-dof if it is not
      // yet (only while small: an explicit entry costs 4 plan bytes, a run descriptor 48)
      std::vector<Run> out;
      std::vector<std::vector<int>> members;  // 1D runs of each 2D run
      std::map<std::tuple<int, int, int, int>, int> open_aff;
      std::map<std::tuple<int, int, int>, int> open_any;
      auto try_join = [&](int gi, const R1 &q, int d0, int k, bool convert) {
         Run &g = out[gi];
         if ((g.n2 + 1) * g.n1 > 64 || q.c > 8) { return false; }
         const int tt = q.c ? slot(d0, 0) - g.s0[0] : 0;
         bool ok = g.n2 == 1 || tt == g.n2 * g.t2;
         for (int h = 1; h < q.c && ok; h++) { ok = slot(d0, h) - g.s0[h] == tt; }
         if (!ok) { return false; }
         const bool gex = g.d1 == kExplicitDofs, qex = q.d1 == kExplicitDofs;
         const int dd = d0 - g.dof0;
         const bool dofs_ok = !gex && !qex && q.d1 == g.d1 && (g.n2 == 1 || dd == g.n2 * g.d2);
         if (!gex && !dofs_ok)
         {
            if (!convert || g.n1 * g.n2 > 12) { return false; }
            g.d1 = kExplicitDofs;  // the run's dofs come from the entry list from now on
            g.d2 = 0;
         }
         if (g.n2 == 1) { g.t2 = tt; g.d2 = g.d1 == kExplicitDofs ? 0 : dd; }
         g.n2++;
         members[gi].push_back(k);
         return true;
      };
      for (size_t k = 0; k < r1s.size(); k++)
      {
         const R1 &q = r1s[k];
         const int d0 = dofs[q.i0];
         const auto ka = std::make_tuple(q.c, q.n, q.d1, q.t1);
         const auto kb = std::make_tuple(q.c, q.n, q.t1);
         int gi = -1;
         auto ia = open_aff.find(ka);
         if (ia != open_aff.end() && try_join(ia->second, q, d0, (int)k, false)) { gi = ia->second; }
         if (gi < 0)
         {
            auto ib = open_any.find(kb);
            if (ib != open_any.end() && try_join(ib->second, q, d0, (int)k, true)) { gi = ib->second; }
         }
         if (gi < 0)
         {
            Run g{q.n, 1, q.c, d0, q.d1, 0, q.t1, 0, q.i0, {}};
            for (int h = 0; h < q.c; h++) { g.s0.push_back(slot(d0, h)); }
            gi = (int)out.size();
            open_aff[ka] = gi;
            out.push_back(g);
            members.push_back({(int)k});
         }
         open_any[kb] = gi;
      }
      // Run order: by first partial slot (the slot locality of the entry order above) or by
      // smallest dof (neighbouring workgroups of the pass then store neighbouring y lines: C5
      // pass -10%, profiles/r3_ab_runorder.txt).  Which one is decided by the 128-B lines (y
      // lines written + partial-slot lines read) that windows of 256 consecutive entries touch,
      // the smaller total wins; ECM2_RUN_ORDER=slot|dof forces one.
      std::vector<size_t> by_slot(out.size()), by_dof;
      for (size_t g = 0; g < out.size(); g++) { by_slot[g] = g; }
      {
         std::vector<long> kmin(out.size(), LONG_MAX);
         for (size_t g = 0; g < out.size(); g++)
            for (int k : members[g])
               for (int j = 0; j < r1s[k].n; j++) { kmin[g] = std::min<long>(kmin[g], dofs[r1s[k].i0 + j]); }
         by_dof = by_slot;
         std::stable_sort(by_dof.begin(), by_dof.end(), [&](size_t a, size_t b) { return kmin[a] < kmin[b]; });
      }
      auto lines_touched = [&](const std::vector<size_t> &go) {
         long total = 0;
         int in_window = 0;
         std::vector<long> ids;
         auto flush = [&] {
            std::sort(ids.begin(), ids.end());
            total += std::unique(ids.begin(), ids.end()) - ids.begin();
            ids.clear();
            in_window = 0;
         };
         for (size_t g : go)
            for (int k : members[g])
               for (int j = 0; j < r1s[k].n; j++)
               {
                  const int d = dofs[r1s[k].i0 + j];
                  ids.push_back((long)d >> 4);
                  for (int h = 0; h < cnt(d); h++) { ids.push_back((1l << 40) + (slot(d, h) >> 4)); }
                  if (++in_window == 256) { flush(); }
               }
         flush();
         return total;
      };
      // chain order: greedy, each next run the unplaced one sharing the most 128-B lines with the
      // run placed last (ties and dead ends: the next unplaced run in slot order), so a face's edge
      // runs follow its interior run and reuse its partial lines while they are in L2
      auto chain_order = [&]() {
         const size_t nr = out.size();
         std::vector<std::vector<long>> rl(nr);
         std::vector<long> all;
         for (size_t g = 0; g < nr; g++)
         {
            for (int k : members[g])
               for (int j = 0; j < r1s[k].n; j++)
               {
                  const int d = dofs[r1s[k].i0 + j];
                  rl[g].push_back((long)d >> 4);
                  for (int h = 0; h < cnt(d); h++) { rl[g].push_back((1l << 40) + (slot(d, h) >> 4)); }
               }
            std::sort(rl[g].begin(), rl[g].end());
            rl[g].erase(std::unique(rl[g].begin(), rl[g].end()), rl[g].end());
            all.insert(all.end(), rl[g].begin(), rl[g].end());
         }
         std::sort(all.begin(), all.end());
         all.erase(std::unique(all.begin(), all.end()), all.end());
         // line -> runs (CSR)
         std::vector<int> loff(all.size() + 1, 0), lrun;
         auto lid = [&](long v) { return (size_t)(std::lower_bound(all.begin(), all.end(), v) - all.begin()); };
         std::vector<std::vector<int>> rli(nr);
         for (size_t g = 0; g < nr; g++)
            for (long v : rl[g])
            {
               const size_t i = lid(v);
               rli[g].push_back((int)i);
               loff[i + 1]++;
            }
         for (size_t i = 0; i < all.size(); i++) { loff[i + 1] += loff[i]; }
         lrun.resize(loff.back());
         {
            std::vector<int> fill(loff.begin(), loff.end() - 1);
            for (size_t g = 0; g < nr; g++)
               for (int i : rli[g]) { lrun[fill[i]++] = (int)g; }
         }
         std::vector<char> placed(nr, 0);
         std::vector<int> shared(nr, 0), touched;
         std::vector<size_t> go;
         go.reserve(nr);
         size_t next_free = 0, cur = 0;
         while (go.size() < nr)
         {
            if (go.empty() || placed[cur])
            {
               while (placed[next_free]) { next_free++; }
               cur = next_free;
            }
            placed[cur] = 1;
            go.push_back(cur);
            size_t best = nr;
            int bs = 0;
            for (int i : rli[cur])
               for (int q = loff[i]; q < loff[i + 1]; q++)
               {
                  const int g = lrun[q];
                  if (placed[g]) { continue; }
                  if (!shared[g]) { touched.push_back(g); }
                  shared[g]++;
               }
            for (int g : touched)
            {
               if (shared[g] > bs || (shared[g] == bs && (size_t)g < best)) { bs = shared[g]; best = g; }
               shared[g] = 0;
            }
            touched.clear();
            cur = best < nr ? best : cur;  // cur placed: the next free run in slot order
         }
         return go;
      };
      const char *ro = std::getenv("ECM2_RUN_ORDER");
      std::vector<size_t> by_chain;
      int pick = 0;  // 0 slot, 1 dof, 2 chain
      if (ro && std::string(ro) == "slot") { pick = 0; }
      else if (ro && std::string(ro) == "dof") { pick = 1; }
      else if (ro && std::string(ro) == "chain") { pick = 2; by_chain = chain_order(); }
      else
      {
         by_chain = chain_order();
         const long ls = lines_touched(by_slot), ld = lines_touched(by_dof), lc = lines_touched(by_chain);
         pick = ld < ls ? 1 : 0;
         if (lc < std::min(ls, ld)) { pick = 2; }
         if (std::getenv("ECM2_PLAN_DUMP"))
         {
            std::fprintf(stderr, "plan range %d: lines touched by slot order %ld, dof order %ld, chain order %ld -> %s\n",
                         range, ls, ld, lc, pick == 2 ? "chain" : pick ? "dof" : "slot");
         }
      }
      const std::vector<size_t> &gord = pick == 2 ? by_chain : pick ? by_dof : by_slot;
      for (size_t g : gord)
      {
         out[g].first = (int)order.size();
         for (int k : members[g])
            for (int j = 0; j < r1s[k].n; j++) { order.push_back(dofs[r1s[k].i0 + j]); }
         runs.push_back(std::move(out[g]));
      }
      ECM2_VERIFY((int)order.size() == r1, ERR_INTERNAL, "run plan lost entries");
   }
   if (std::getenv("ECM2_PLAN_DUMP"))  // (diagnostic) run classes of the summation plan
   {
      std::map<std::tuple<int, int, int, int>, std::pair<long, long>> h;
      for (const Run &g : runs)
      {
         auto &v = h[std::make_tuple(g.d1 == kExplicitDofs, g.c, g.n1, g.n2)];
         v.first++;
         v.second += (long)g.n1 * g.n2;
      }
      std::vector<std::pair<long, std::tuple<int, int, int, int>>> top;
      for (auto &kv : h) { top.push_back({kv.second.first, kv.first}); }
      std::sort(top.rbegin(), top.rend());
      std::fprintf(stderr, "plan: %zu runs, %d entries\n", runs.size(), n_sh_);
      for (size_t i = 0; i < top.size() && i < 30; i++)
      {
         const auto &k = top[i].second;
         std::fprintf(stderr, "  explicit %d holders %d shape %dx%d: %ld runs, %ld entries\n", std::get<0>(k),
                      std::get<1>(k), std::get<2>(k), std::get<3>(k), top[i].first, h[k].second);
      }
   }
   std::vector<int> rdesc, rslots, blocks;
   rdesc.reserve((runs.size() + 1) * 12);
   for (const Run &g : runs)
   {
      // every entry of the run must be what the descriptor computes (checked, host side)
      for (int j = 0; j < g.n1 * g.n2; j++)
      {
         const int a = j % g.n1, b = j / g.n1, d = order[g.first + j];
         bool ok = (g.d1 == kExplicitDofs || d == g.dof0 + a * g.d1 + b * g.d2) && cnt(d) == g.c;
         for (int h = 0; h < g.c && ok; h++) { ok = slot(d, h) == g.s0[h] + a * g.t1 + b * g.t2; }
         ECM2_VERIFY(ok, ERR_INTERNAL, "run plan entry " << g.first + j << " does not match its run");
      }
      const bool ex = g.d1 == kExplicitDofs;  // shape bit 24: dofs from the entry list
      ECM2_VERIFY(g.c < 256, ERR_UNSUPPORTED, "a dof with " << g.c << " holders");
      int row[12] = {g.n1 | g.n2 << 8 | g.c << 16 | (ex ? 1 << 24 : 0), g.dof0, ex ? 0 : g.d1, ex ? 0 : g.d2,
                     g.t1, g.t2, g.first, (int)rslots.size(), 0, 0, 0, 0};
      for (int h = 0; h < g.c; h++)
      {
         if (h < 4) { row[8 + h] = g.s0[h]; }
         rslots.push_back(g.s0[h]);
      }
      rdesc.insert(rdesc.end(), row, row + 12);
   }
   const int sentinel[12] = {1, 0, 0, 0, 0, 0, n_sh_, 0, 0, 0, 0, 0};
   rdesc.insert(rdesc.end(), sentinel, sentinel + 12);
   // blocks: whole runs, <= 256 entries each, never across the owned / ghost boundary
   sh_nblk_owned_ = 0;
   for (size_t r = 0; r < runs.size();)
   {
      const bool ghost = runs[r].first >= n_sh_owned_;
      size_t e = r;
      int n = 0;
      while (e < runs.size() && (runs[e].first >= n_sh_owned_) == ghost && n + runs[e].n1 * runs[e].n2 <= 256)
      {
         n += runs[e].n1 * runs[e].n2;
         e++;
      }
      bool ex = false;
      for (size_t g = r; g < e; g++) { ex = ex || runs[g].d1 == kExplicitDofs; }
      blocks.push_back((int)r);
      blocks.push_back((int)e);
      blocks.push_back(runs[r].first);
      blocks.push_back(n | (ex ? 1 << 30 : 0));
      if (!ghost) { sh_nblk_owned_++; }
      r = e;
   }
   sh_nblk_ = (int)blocks.size() / 4;
   n_runs_ = (long)runs.size();
   sh_runs_.upload(rdesc, s);
   sh_rslots_.upload(rslots.empty() ? std::vector<int>{0} : rslots, s);
   sh_blocks_.upload(blocks.empty() ? std::vector<int>{0, 0, 0, 0} : blocks, s);
   n_explicit_runs_ = 0;
   for (const Run &g : runs) { n_explicit_runs_ += g.d1 == kExplicitDofs; }
   sh_pdof_.upload(order.empty() ? std::vector<int>{0} : order, s);
}

void PAForm::set_kernel(int mode)
{
   ECM2_VERIFY(mode >= KERNEL_AUTO && mode <= KERNEL_LINE, ERR_ARG, "unknown kernel mode " << mode);
   mode_ = mode;
   gmap_blk_.resize(0);   // the scatter plan belongs to one fused kernel: rebuild it
   gmap_line_.resize(0);
   assembled_ = false;
}

static bool has_tpe(int D, int Q) { return (D == 2 && Q == 3) || (D == 3 && Q == 4); }

void PAForm::assemble(hipStream_t s)
{
   ECM2_VERIFY(enodes_.size() || jac_ || ne_ == 0, ERR_STATE, "assemble: no geometry set");
   resolved_mode_ = mode_;
   if (mode_ == KERNEL_AUTO)
   {
      resolved_mode_ = has_tpe(D_, Q_) ? KERNEL_TPE : (kern::has_line(D_, Q_) ? KERNEL_LINE : KERNEL_WPE);
   }
   ECM2_VERIFY(resolved_mode_ != KERNEL_TPE || has_tpe(D_, Q_), ERR_UNSUPPORTED,
               "thread-per-element kernel needs (D1D,Q1D) in {(2,3),(3,4)}");
   ECM2_VERIFY(resolved_mode_ != KERNEL_LINE || kern::has_line(D_, Q_), ERR_UNSUPPORTED,
               "line kernel needs Q1D in {D1D, D1D+1} and Q1D <= 8");
   // a general (nonsymmetric) matrix coefficient: the reference's 9-entry qdata (NATIVE9), read by
   // the workgroup-per-element kernels; any other vector / matrix coefficient keeps 6 symmetric
   // entries but varies per point in direction: no geometry compression
   const int cdim = have_diff_ ? cdiff_.dim() : 1;
   if (cdim == 9)
   {
      ECM2_VERIFY(mode_ == KERNEL_AUTO || mode_ == KERNEL_WPE || mode_ == KERNEL_UNFUSED, ERR_UNSUPPORTED,
                  "a general matrix coefficient runs the workgroup-per-element or unfused kernels");
      if (mode_ == KERNEL_AUTO) { resolved_mode_ = KERNEL_WPE; }
   }
   layout_.kind = (resolved_mode_ == KERNEL_TPE) ? QLAYOUT_BLOCKED : (cdim == 9 ? QLAYOUT_NATIVE9 : QLAYOUT_NATIVE);
   layout_.pw = 2;
   // Compressed geometry for the fused kernels (thread-per-element p <= 2: AFFINE / TRILINEAR;
   // line / brick p >= 3: AFFINE_E / TRILINEAR_E), with both integrators or a diffusion-only form
   // such as ex16's K (point values W beta [/ det J] alone, 8 B per point).  A mass-only form keeps
   // the mass stream, already one 8-byte W alpha det J per point.
   const bool fused = resolved_mode_ == KERNEL_TPE || resolved_mode_ == KERNEL_LINE;
   const bool comp = compress_ && have_diff_ && cdim == 1 && fused;
   const bool tpe = resolved_mode_ == KERNEL_TPE;
   bool affine = affine_;
   if (jac_ && comp)
   {
      affine = kern::jacobians_affine(ne_, NQ_, jac_, s);  // the reference binding's geometry
   }
   if (affine && comp)
   {
      layout_.kind = tpe ? QLAYOUT_AFFINE : QLAYOUT_AFFINE_E;
      layout_.pw = have_mass_ ? 2 : 1;
   }
   else if (!affine && comp)
   {
      // general trilinear hexes: the map coefficients per element (from the corners, or fitted
      // to the reference binding's Jacobians when they are a trilinear map's), J per point
      bool tl = !jac_ && enodes_.size();
      if (jac_)
      {
         QPts qp = {};
         for (int q = 0; q < Q_ && q < MAX_Q1D; q++) { qp.x[q] = maps_.qpts[q]; }
         cfit_.resize(std::max(1, ne_) * 21);
         tl = kern::jacobians_trilinear_fit(ne_, Q_, qp, jac_, cfit_.data(), s);
      }
      if (tl)
      {
         layout_.kind = tpe ? QLAYOUT_TRILINEAR : QLAYOUT_TRILINEAR_E;
         layout_.pw = have_mass_ ? 2 : 1;
      }
   }

   // the merge plan (cross-wave faces), the regular blocks and the partial-slot layout belong
   // to the qdata layout they were built for
   if (gmap_blk_.size() && plan_kind_ != layout_.kind) { gmap_blk_.resize(0); }
   if (resolved_mode_ == KERNEL_TPE && !gmap_blk_.size() && ne_ > 0)
   {
      plan_kind_ = layout_.kind;
      if (perm_host_.empty())
      {
         // no caller order: 4x4x4 face-linked bricks first (one per wave), per apply segment
         std::vector<int> cuts{0};
         for (int sp : splits_) { cuts.push_back(std::min(ne_, sp * kElemBlock)); }
         cuts.push_back(ne_);
         std::sort(cuts.begin(), cuts.end());
         for (size_t k = 0; k + 1 < cuts.size(); k++)
         {
            const int e0 = cuts[k], n = cuts[k + 1] - cuts[k];
            if (n <= 0) { continue; }
            std::vector<int> sub(gmap_host_.begin() + (size_t)e0 * ND_, gmap_host_.begin() + (size_t)(e0 + n) * ND_);
            for (int e : face_brick_order(n, D_, sub)) { perm_host_.push_back(e0 + e); }
         }
         perm_auto_ = true;
      }
      const int nblk = layout_.nblk();
      std::vector<int> gint((size_t)ne_ * ND_), pos(ne_);
      for (int i = 0; i < ne_; i++)
      {
         const int e = perm_host_.empty() ? i : perm_host_[i];
         pos[e] = i;
         std::copy(&gmap_host_[(size_t)e * ND_], &gmap_host_[(size_t)e * ND_] + ND_, &gint[(size_t)i * ND_]);
      }
      ECM2_VERIFY(ndofs_ < (1 << 30), ERR_UNSUPPORTED, "fused kernel supports < 2^30 dofs");
      ECM2_VERIFY((size_t)nblk * ND_ * 64 < (1ull << 31), ERR_UNSUPPORTED, "too many elements for int slots");
      std::vector<char> holds;
      std::vector<int> fl, hcount;
      // workgroups as the launches group them (4 blocks from each apply segment's start);
      // waves of a workgroup may assemble shared faces through LDS (AFFINE kernels), except
      // in segments launched with the one-block-per-workgroup latency kernel
      std::vector<std::array<int, 3>> groups;
      {
         std::vector<int> seg{0, nblk};
         for (int sp : splits_) { seg.push_back(std::max(0, std::min(nblk, sp))); }
         std::sort(seg.begin(), seg.end());
         seg.erase(std::unique(seg.begin(), seg.end()), seg.end());
         const bool xw = layout_.kind == QLAYOUT_AFFINE || layout_.kind == QLAYOUT_TRILINEAR;
         for (size_t k = 0; k + 1 < seg.size(); k++)
         {
            const bool lat = latency_from_ >= 0 && seg[k] >= latency_from_;
            for (int b = seg[k]; b < seg[k + 1]; b += 4)
            {
               groups.push_back({b, std::min(b + 4, seg[k + 1]), (xw && !lat) ? 1 : 0});
            }
         }
      }
      build_merge_plan(ne_, D_, gint, ndofs_, holds, hcount, fl, groups);
      // blocked map: dof | shared << 30 | sign << 31
      std::vector<int> blk((size_t)nblk * ND_ * 64, 0);
      for (int i = 0; i < ne_; i++)
      {
         const int b = i / 64, l = i % 64;
         for (int a = 0; a < ND_; a++)
         {
            const int g = gint[(size_t)i * ND_ + a];
            const unsigned d = (unsigned)(g >= 0 ? g : -1 - g);
            const unsigned enc = d | ((hcount[d] > 1 ? 1u : 0u) << 30) | ((g < 0 ? 1u : 0u) << 31);
            blk[((size_t)b * ND_ + a) * 64 + l] = (int)enc;
         }
      }
      // Regular blocks (the AFFINE kernel): the block's 64 elements a 4x4x4 lattice brick
      // (lane = ex + 4 ey + 16 ez) of a lattice-numbered region, d = base + X sx + Y sy + Z sz on
      // the block's (4(D-1)+1)^3 lattice, every dof owned, no orientation signs, and the held
      // shared dofs exactly those on the block faces a 6-bit mask names.  The kernel then reads
      // 5 ints per block instead of 64 ND map entries (C4: 136 MB per Mult and a dependent load
      // chain at the gather and the store).  Decided per block (a partitioned rank's interior
      // blocks are regular, its boundary blocks are not); treg_all when every block is.
      treg_.resize(0);
      treg_all_ = false;
      tlat_all_ = false;
      n_treg_ = 0;
      n_tlat_ = 0;
      lmap_.resize(0);
      const int ns = tpe_surface_points(D_);
      std::vector<char> breg_ok(nblk, 0);
      if (layout_.kind == QLAYOUT_AFFINE || layout_.kind == QLAYOUT_TRILINEAR)
      {
         const int L = 4 * (D_ - 1);
         std::vector<int> reg((size_t)nblk * 8, 0);
         auto ent = [&](int b, int l, int a) { return blk[((size_t)b * ND_ + a) * 64 + l]; };
         auto faces = [&](int X, int Y, int Z) {
            return (X == 0) | (X == L) << 1 | (Y == 0) << 2 | (Y == L) << 3 | (Z == 0) << 4 | (Z == L) << 5;
         };
         int nreg = 0;
         for (int b = 0; b < nblk; b++)
         {
            // (blocks the latency kernel applies store [a][lane] slots: never regular)
            bool regular = (long)(b + 1) * 64 <= ne_ && (latency_from_ < 0 || b < latency_from_);
            auto dv = [&](int l, int a) { return ent(b, l, a) & 0x3fffffff; };
            const int base = dv(0, 0), sx = dv(0, 1) - base, sy = dv(0, D_) - base, sz = dv(0, D_ * D_) - base;
            int mask = 0;
            for (int l = 0; l < 64 && regular; l++)
               for (int a = 0; a < ND_ && regular; a++)
               {
                  const int X = (D_ - 1) * (l & 3) + a % D_, Y = (D_ - 1) * ((l >> 2) & 3) + (a / D_) % D_,
                            Z = (D_ - 1) * (l >> 4) + a / (D_ * D_);
                  const unsigned g = (unsigned)ent(b, l, a);
                  const int d = (int)(g & 0x3fffffffu);
                  regular = !(g >> 31) && d < n_owned_ && d == base + X * sx + Y * sy + Z * sz;
                  // a held entry on exactly one face sets that face's bit
                  const int f = faces(X, Y, Z);
                  if (regular && holds[((size_t)b * 64 + l) * ND_ + a] && f && !(f & (f - 1)) && hcount[d] > 1)
                  {
                     mask |= f;
                  }
               }
            for (int l = 0; l < 64 && regular; l++)
               for (int a = 0; a < ND_ && regular; a++)
               {
                  if (!holds[((size_t)b * 64 + l) * ND_ + a]) { continue; }
                  const int X = (D_ - 1) * (l & 3) + a % D_, Y = (D_ - 1) * ((l >> 2) & 3) + (a / D_) % D_,
                            Z = (D_ - 1) * (l >> 4) + a / (D_ * D_);
                  regular = (hcount[dv(l, a)] > 1) == ((faces(X, Y, Z) & mask) != 0);
               }
            if (!regular) { continue; }
            int *r = &reg[(size_t)b * 8];
            r[0] = base; r[1] = sx; r[2] = sy; r[3] = sz; r[4] = mask; r[7] = 1;
            breg_ok[b] = 1;
            nreg++;
         }
         n_treg_ = nreg;
         // Lattice-slot blocks (flag 2): complete blocks whose dofs are not a lattice (the
         // reference's entity numbering) but whose held shared entries all sit on distinct points
         // of the block surface: their partial slots are face-grouped like a regular block's, so
         // the summation plan's runs stay long (with the dofs from its entry list)
         // Their dofs come from a block lattice map (tpe_lattice_slot order, one entry per lattice
         // point): every entry of the block at one lattice point must encode the same dof, none
         // with an orientation sign.
         int nlat = 0;
         const int NL = tpe_lattice_points(D_);
         std::vector<int> lmap;
         for (int b = 0; b < nblk; b++)
         {
            if (breg_ok[b] || (long)(b + 1) * 64 > ne_ || (latency_from_ >= 0 && b >= latency_from_)) { continue; }
            std::vector<char> used(ns, 0);
            std::vector<int> lm(NL, -1);
            bool ok = true;
            for (int l = 0; l < 64 && ok; l++)
               for (int a = 0; a < ND_ && ok; a++)
               {
                  const int X = (D_ - 1) * (l & 3) + a % D_, Y = (D_ - 1) * ((l >> 2) & 3) + (a / D_) % D_,
                            Z = (D_ - 1) * (l >> 4) + a / (D_ * D_);
                  const int g = blk[((size_t)b * ND_ + a) * 64 + l];
                  int &m = lm[tpe_lattice_slot(D_, X, Y, Z)];
                  ok = !((unsigned)g >> 31) && (m < 0 || m == g);
                  m = g;
               }
            for (int l = 0; l < 64 && ok; l++)
               for (int a = 0; a < ND_ && ok; a++)
               {
                  if (!holds[((size_t)b * 64 + l) * ND_ + a]) { continue; }
                  if (hcount[blk[((size_t)b * ND_ + a) * 64 + l] & 0x3fffffff] <= 1) { continue; }
                  const int X = (D_ - 1) * (l & 3) + a % D_, Y = (D_ - 1) * ((l >> 2) & 3) + (a / D_) % D_,
                            Z = (D_ - 1) * (l >> 4) + a / (D_ * D_);
                  const int si = tpe_surface_index(D_, X, Y, Z);
                  ok = si >= 0 && !used[si];
                  if (ok) { used[si] = 1; }
               }
            if (!ok) { continue; }
            reg[(size_t)b * 8 + 7] = 2;
            breg_ok[b] = 2;
            nlat++;
            if (lmap.empty()) { lmap.assign((size_t)nblk * NL, 0); }
            std::copy(lm.begin(), lm.end(), lmap.begin() + (size_t)b * NL);
         }
         n_tlat_ = nlat;
         lmap_.resize(0);
         if (nlat) { lmap_.upload(lmap, s); }
         if (nreg || nlat)
         {
            treg_.upload(reg, s);
            treg_all_ = nreg == nblk && (latency_from_ < 0 || latency_from_ >= nblk);
            tlat_all_ = nlat == nblk && (latency_from_ < 0 || latency_from_ >= nblk);
         }
      }
      part_stride_ = treg_all_ || tlat_all_ ? ns : ND_ * 64;
      {
         // partial slots: [blk][a][lane]; on regular blocks [blk][face-grouped surface index of
         // the block lattice] (tpe_surface_index: a face's two holders list it at the same
         // offset, so the summation pass reads both holders' runs contiguously)
         std::vector<int> hdof, hslot;
         for (int b = 0; b < nblk; b++)
            for (int a = 0; a < ND_; a++)
               for (int l = 0; l < 64; l++)
               {
                  if (!holds[((size_t)b * 64 + l) * ND_ + a]) { continue; }
                  const int d = blk[((size_t)b * ND_ + a) * 64 + l] & 0x3fffffff;
                  if (hcount[d] > 1)
                  {
                     hdof.push_back(d);
                     if (breg_ok[b])
                     {
                        const int X = (D_ - 1) * (l & 3) + a % D_, Y = (D_ - 1) * ((l >> 2) & 3) + (a / D_) % D_,
                                  Z = (D_ - 1) * (l >> 4) + a / (D_ * D_);
                        const int si = tpe_surface_index(D_, X, Y, Z);
                        ECM2_VERIFY(si >= 0, ERR_INTERNAL, "block " << b << ": interior lattice point shared");  // (checked)
                        hslot.push_back(b * part_stride_ + si);
                     }
                     else { hslot.push_back(b * part_stride_ + a * 64 + l); }
                  }
               }
         // the plan wants each dof's holders in ascending slot order
         std::vector<size_t> ord(hslot.size());
         for (size_t i = 0; i < ord.size(); i++) { ord[i] = i; }
         std::sort(ord.begin(), ord.end(), [&](size_t p, size_t q) { return hslot[p] < hslot[q]; });
         std::vector<int> hd(ord.size()), hs(ord.size());
         for (size_t i = 0; i < ord.size(); i++) { hd[i] = hdof[ord[i]]; hs[i] = hslot[ord[i]]; }
         build_shared_plan(hcount, hd, hs, s);
      }
      gmap_blk_.upload(blk, s);
      lane_flags_.upload(fl, s);
      pos_.upload(pos, s);
      std::vector<int> perm(ne_);
      for (int e = 0; e < ne_; e++) { perm[pos[e]] = e; }
      perm_dev_.upload(perm, s);
      rowtab_.upload(kern::make_row_table(maps_), s);
      drowtab_.upload(kern::make_diag_row_table(maps_), s);
      ECM2_HIP(hipStreamSynchronize(s));
   }
   if (!btab_.size())
   {
      const BasisDev bd = make_basis_dev(basis_, D_, Q_);
      btab_.upload(&bd, 1, s);
   }
   if (resolved_mode_ == KERNEL_LINE && !gmap_line_.size() && ne_ > 0)
   {
      // Bricks of 2 x 2 x bz elements (deterministic scatter, both integrators) take every
      // element they can; the leftovers run the per-element line kernel, listed per
      // 64-element block (apply_blocks ranges map to list ranges).  Then the encoded maps and
      // the deterministic-scatter plan over the holding entries: the bricks' lattice points,
      // the leftovers' entries.
      ECM2_VERIFY(ndofs_ < (1 << 30), ERR_UNSUPPORTED, "fused kernel supports < 2^30 dofs");
      ECM2_VERIFY((size_t)ne_ * ND_ < (1ull << 31) && ne_ < (1 << 24), ERR_UNSUPPORTED,
                  "too many elements for the line kernel's chunk table");
      auto dofv = [](int g) { return g >= 0 ? g : -1 - g; };
      const int nblk = layout_.nblk();
      // default 2 x 2 x 1 (C5, profiles/ab_brick.sh: 0.861 ms against 1.018 ms per element and
      // 1.114 ms for 2 x 2 x 2)
      int bz = (scatter_ == SCATTER_PARTIALS && have_mass_ && have_diff_) ? (line_bricks_ >= 0 ? line_bricks_ : 1) : 0;
      if (bz == 2 && !kern::has_brick(D_, Q_, 2)) { bz = 1; }
      if (bz == 1 && !kern::has_brick(D_, Q_, 1)) { bz = 0; }
      std::vector<int> belem;
      std::vector<char> in_brick(ne_, 0);
      if (bz)
      {
         std::vector<int> seg(ne_, 0);
         for (int e = 0; e < ne_; e++)
         {
            for (int sp : splits_) { seg[e] += (e / kElemBlock >= sp); }
         }
         find_bricks(ne_, D_, gmap_host_, bz, seg, belem, in_brick);
      }
      const int nbe = 4 * (bz ? bz : 1);
      n_bricks_ = bz ? (int)(belem.size() / nbe) : 0;
      brick_bz_ = n_bricks_ ? bz : 0;
      brick_np_ = brick_bz_ ? kern::brick_points(D_, brick_bz_) : 0;
      const int LX = 2 * D_ - 1, LY = LX;
      // lattice map of each brick (dof per lattice point; internal faces coincide by construction)
      std::vector<int> bdof((size_t)n_bricks_ * brick_np_, -1);
      for (int k = 0; k < n_bricks_; k++)
         for (int elt = 0; elt < nbe; elt++)
         {
            const int e = belem[(size_t)k * nbe + elt], ex = elt & 1, ey = (elt >> 1) & 1, ez = elt >> 2;
            for (int dz = 0; dz < D_; dz++)
               for (int dy = 0; dy < D_; dy++)
                  for (int dx = 0; dx < D_; dx++)
                  {
                     const int p = ((ez * (D_ - 1) + dz) * LY + ey * (D_ - 1) + dy) * LX + ex * (D_ - 1) + dx;
                     const int d = dofv(gmap_host_[(size_t)e * ND_ + (dz * D_ + dy) * D_ + dx]);
                     int &b = bdof[(size_t)k * brick_np_ + p];
                     ECM2_VERIFY(b < 0 || b == d, ERR_INTERNAL, "brick " << k << " lattice point " << p
                                                                    << " holds two dofs");
                     b = d;
                  }
         }
      std::vector<int> lelem, coff(nblk + 1, 0), boff(nblk + 1, 0);
      std::vector<char> holds((size_t)ne_ * ND_, 0);
      for (int bk = 0; bk < nblk; bk++)
      {
         for (int e = bk * 64; e < std::min(ne_, bk * 64 + 64); e++)
         {
            if (in_brick[e]) { continue; }
            lelem.push_back(e);
            for (int a = 0; a < ND_; a++) { holds[(size_t)e * ND_ + a] = 1; }
         }
         coff[bk + 1] = (int)lelem.size();
      }
      const int n_left = (int)lelem.size();
      for (int k = 0, bk = 0; bk < nblk; bk++)
      {
         while (k < n_bricks_ && belem[(size_t)k * nbe] / kElemBlock == bk) { k++; }
         boff[bk + 1] = k;
      }
      ECM2_VERIFY(boff[nblk] == n_bricks_, ERR_INTERNAL, "bricks not ordered by first element");
      std::vector<int> hcount(ndofs_, 0);
      for (int d : bdof) { hcount[d]++; }
      for (size_t i = 0; i < gmap_host_.size(); i++) { if (holds[i]) { hcount[dofv(gmap_host_[i])]++; } }
      auto encode = [&](int d, bool neg) {
         return (int)((unsigned)d | ((hcount[d] > 1 ? 1u : 0u) << 30) | ((neg ? 1u : 0u) << 31));
      };
      // brick partial slots: [brick][face-grouped surface index]; only surface points can be
      // shared (a brick holds its interior lattice points alone: checked)
      const int nsurf = brick_bz_ ? brick_surface_points(D_, brick_bz_) : 0;
      part_line_off_ = (long)n_bricks_ * nsurf;
      std::vector<int> enc(gmap_host_.size()), benc(bdof.size()), hdof, hslot;
      std::vector<long> bslot;
      for (size_t i = 0; i < bdof.size(); i++)
      {
         benc[i] = encode(bdof[i], false);
         if (hcount[bdof[i]] > 1)
         {
            const int k = (int)(i / brick_np_), p = (int)(i % brick_np_);
            const int si = brick_surface_index(D_, brick_bz_, p % LX, (p / LX) % LY, p / (LX * LY));
            ECM2_VERIFY(si >= 0, ERR_INTERNAL, "brick " << k << ": interior lattice point " << p << " is shared");
            hdof.push_back(bdof[i]);
            bslot.push_back((long)k * nsurf + si);
         }
      }
      // the plan wants the holders in ascending slot order
      {
         std::vector<size_t> ord(bslot.size());
         for (size_t i = 0; i < ord.size(); i++) { ord[i] = i; }
         std::sort(ord.begin(), ord.end(), [&](size_t a, size_t b) { return bslot[a] < bslot[b]; });
         std::vector<int> hd(ord.size());
         hslot.resize(ord.size());
         for (size_t i = 0; i < ord.size(); i++)
         {
            hd[i] = hdof[ord[i]];
            hslot[i] = (int)bslot[ord[i]];
         }
         hdof.swap(hd);
      }
      ECM2_VERIFY(part_line_off_ + (long)nblk * ND_ * 64 < (1l << 31), ERR_UNSUPPORTED, "too many partial slots");
      for (size_t i = 0; i < gmap_host_.size(); i++)
      {
         const int g = gmap_host_[i];
         const int d = dofv(g);
         enc[i] = encode(d, g < 0);
         if (holds[i] && hcount[d] > 1)
         {
            hdof.push_back(d);
            hslot.push_back((int)(part_line_off_ + (long)i));
         }
      }
      build_shared_plan(hcount, hdof, hslot, s);
      // Regular bricks: every brick's lattice map an affine function of the lattice point
      // (d = base + X sx + Y sy + Z sz, a lattice-numbered mesh) and its shared points exactly
      // those on the brick faces other holders touch (one face-mask bit per face) -- the kernel
      // then computes dofs and shared flags from 5 ints per brick instead of reading the map
      breg_.resize(0);
      if (n_bricks_ && n_owned_ == ndofs_)
      {
         const int LZ = brick_bz_ * (D_ - 1) + 1;
         std::vector<int> reg((size_t)n_bricks_ * 8, 0);
         bool regular = true;
         for (int k = 0; k < n_bricks_ && regular; k++)
         {
            const int *b = &bdof[(size_t)k * brick_np_];
            const int base = b[0], sx = b[1] - base, sy = b[LX] - base, sz = b[LX * LY] - base;
            auto faces = [&](int X, int Y, int Z) {
               return (X == 0) | (X == LX - 1) << 1 | (Y == 0) << 2 | (Y == LY - 1) << 3 | (Z == 0) << 4 |
                      (Z == LZ - 1) << 5;
            };
            // face bit = sharing of a point inside that face (on no other face)
            const int cx = LX / 2, cy = LY / 2, cz = LZ / 2;
            const int probe[6][3] = {{0, cy, cz}, {LX - 1, cy, cz}, {cx, 0, cz}, {cx, LY - 1, cz}, {cx, cy, 0}, {cx, cy, LZ - 1}};
            int mask = 0;
            for (int f = 0; f < 6; f++)
            {
               const int p = (probe[f][2] * LY + probe[f][1]) * LX + probe[f][0];
               if (hcount[b[p]] > 1) { mask |= 1 << f; }
            }
            for (int p = 0; p < brick_np_ && regular; p++)
            {
               const int X = p % LX, Y = (p / LX) % LY, Z = p / (LX * LY);
               regular = b[p] == base + X * sx + Y * sy + Z * sz &&
                         (hcount[b[p]] > 1) == ((faces(X, Y, Z) & mask) != 0);
            }
            int *r = &reg[(size_t)k * 8];
            r[0] = base; r[1] = sx; r[2] = sy; r[3] = sz; r[4] = mask;
         }
         if (regular) { breg_.upload(reg, s); }
      }
      gmap_line_.upload(enc, s);
      lelem_.upload(lelem.empty() ? std::vector<int>{0} : lelem, s);
      lelem_off_ = coff;
      belem_.upload(belem, s);
      bmap_.upload(benc, s);
      brick_off_ = boff;
      n_left_ = n_left;
      ECM2_HIP(hipStreamSynchronize(s));
   }
   layout_.pos = layout_.blocked() ? pos_.data() : nullptr;
   layout_.perm = layout_.blocked() ? perm_dev_.data() : nullptr;
   if (!use_partials()) { part_.resize(0); }
   else if (resolved_mode_ == KERNEL_LINE)
   {
      // [bricks' lattice slots | leftover elements' [e][nd] slots (when there are any)]
      part_.resize(std::max<size_t>(1, (size_t)part_line_off_ + (n_left_ ? (size_t)ne_ * ND_ : 0)));
   }
   else { part_.resize((size_t)layout_.nblk() * part_stride_); }
   // Coefficient snapshot (k_apply_tpe_ts): the diffusion coefficient a law of an H1 field on this
   // space (GridFunctionCoefficient, AffineGridFunctionCoefficient, the perfusion law), AFFINE
   // geometry, p = 2, every block a lattice brick, no attribute marker on the diffusion integrator.
   // The mass then streams W alpha det J per point (tmass 1), or nothing per point when its
   // coefficient is a constant or a law of the same field (tmass 2: (c alpha) det J per element).
   layout_.tsnap = 0;
   layout_.tmass = 0;
   layout_.tlaw = 0;
   tsnap_.resize(0);
   // (p >= 3: the same snapshot in the brick kernel was measured and rejected, profiles/r5/ab_c5*.txt)
   const bool ts_tpe = layout_.kind == QLAYOUT_AFFINE && resolved_mode_ == KERNEL_TPE && D_ == 3 && Q_ == 4 &&
                       (treg_all_ || tlat_all_);
   if (tsnap_pref_ && ts_tpe && have_diff_ && cdiff_.gridfunc() && cdiff_.lvec && !marked_[INTEG_DIFFUSION])
   {
      layout_.tsnap = 1;
      const bool mass_law = have_mass_ && cmass_.gridfunc() && cmass_.lvec == cdiff_.lvec;
      layout_.tmass = !have_mass_ ? 0 : (cmass_.kind == COEFF_CONSTANT || mass_law) ? 2 : 1;
      layout_.pw = layout_.tmass == 1 ? 1 : 0;
      // an affine (or identity) diffusion law alone is applied to the dofs (the interpolated T' is
      // the law at the point: the basis sums to 1); a nonlinear law, or a mass law of the same field,
      // needs the field itself at the point
      layout_.tlaw = (mass_law || cdiff_.kind == COEFF_GRIDFUNC_PERFUSION) ? 1 : 0;
      // T' = A + B T at every dof, taken here only: the Assemble-time field (the reference's qdata
      // semantics; the diagonal and the qdata export read the same snapshot)
      double A = 0.0, B = 1.0;
      if (!layout_.tlaw && cdiff_.kind == COEFF_GRIDFUNC_AFFINE)
      {
         A = cdiff_.scale * (1.0 - cdiff_.slope * cdiff_.t_ref);
         B = cdiff_.scale * cdiff_.slope;
      }
      if (treg_all_)
      {
         tsnap_.resize(std::max(1, ndofs_));
         kern::affine_snapshot(ndofs_, cdiff_.lvec, A, B, tsnap_.data(), s);
      }
      else
      {
         // lattice-map blocks (the reference's numbering): the snapshot in their lattice-slot order,
         // read contiguously by the kernel (no second dependent gather through the map)
         layout_.tsnap = 2;
         const int nlp = tpe_lattice_points(D_);
         tsnap_.resize((size_t)layout_.nblk() * nlp);
         kern::affine_snapshot_lattice(layout_.nblk(), nlp, lmap_.data(), cdiff_.lvec, A, B, tsnap_.data(), s);
      }
   }
   setup_qdata(s);
   // The marker diagonal's element weights (assemble_diagonal), from the Assemble-time attributes
   // (the reference reads them in SetupRestrictionOperators, bilinearform_ext.cpp:269)
   diag_integ_ = -1;
   diag_w_.resize(0);
   if (order_added_.size() == 2 && marked_[order_added_[1]])
   {
      const int F = order_added_[0], S = order_added_[1];
      const std::vector<double> wf = marker_weights(F), ws = marker_weights(S);
      bool differ = false;
      for (int e = 0; e < ne_ && !differ; e++) { differ = wf[e] != 0.0 && ws[e] == 0.0; }
      if (differ)
      {
         diag_integ_ = F;
         diag_w_.upload(ws, s);
         ECM2_HIP(hipStreamSynchronize(s));  // ws is a host temporary
      }
   }
   assembled_ = true;
   gen_++;
}

std::vector<double> PAForm::marker_weights(int k) const
{
   std::vector<double> w(ne_, 1.0);
   if (!marked_[k]) { return w; }
   ECM2_VERIFY((int)attr_.size() == ne_, ERR_STATE, "a marked integrator needs the element attributes "
                                                    "(ecm2_pa_form_set_attributes)");
   for (int e = 0; e < ne_; e++)
   {
      const int a = attr_[e];
      ECM2_VERIFY(a <= (int)marker_[k].size(), ERR_ARG, "element " << e << " has attribute " << a
                                                         << " beyond the marker's " << marker_[k].size() << " entries");
      w[e] = (a > 0 && marker_[k][a - 1] != 0) ? 1.0 : 0.0;
   }
   return w;
}

const double *PAForm::coeff_points(const CoeffDesc &c, DeviceArray<double> &tmp, hipStream_t s) const
{
   if (c.quad_values()) { return c.quad; }
   if (c.gridfunc())
   {
      tmp.resize((size_t)ne_ * NQ_);
      kern::coeff_gridfunc(ne_, D_, Q_, gmap_.data(), basis_, btab(), c, tmp.data(), s);
      return tmp.data();
   }
   return nullptr;
}

void PAForm::setup_qdata(hipStream_t s)
{
   // (compressed layouts: qd_mass_ holds the point values, present with either integrator)
   const bool comp = layout_.compressed();
   qd_diff_.resize(have_diff_ ? layout_.diff_size() : 0);
   qd_mass_.resize(have_mass_ || comp ? layout_.mass_size() : 0);
   // the setup kernels write every entry except the padding lanes of a partial last block
   // (blocked layout), which are cleared so the apply kernels stream defined values
   if (layout_.blocked() && ne_ % kElemBlock)
   {
      const size_t nb = layout_.nblk();
      if (qd_diff_.size())
      {
         const size_t per = qd_diff_.size() / nb;
         ECM2_HIP(hipMemsetAsync(qd_diff_.data() + (nb - 1) * per, 0, per * sizeof(double), s));
      }
      if (qd_mass_.size())
      {
         const size_t per = qd_mass_.size() / nb;
         ECM2_HIP(hipMemsetAsync(qd_mass_.data() + (nb - 1) * per, 0, per * sizeof(double), s));
      }
   }

   // Attribute markers: per marked integrator, element weights 1 (marker[attr - 1] != 0) or 0,
   // applied to its coefficient at setup (the reference masks the integrator's E-vector output,
   // AddWithMarkers_, bilinearform_ext.cpp:753-774: the same operator)
   for (int k = 0; k < 2; k++)
   {
      CoeffDesc &c = k == INTEG_MASS ? cmass_ : cdiff_;
      c.emask = nullptr;
      if (!(k == INTEG_MASS ? have_mass_ : have_diff_)) { continue; }
      if (!marked_[k]) { continue; }
      std::vector<double> w = marker_weights(k);
      w.resize(std::max(1, ne_));
      emask_[k].upload(w, s);
      ECM2_HIP(hipStreamSynchronize(s));  // w is a host temporary
      c.emask = emask_[k].data();
   }

   // Coefficient values at quadrature points (CoefficientVector::Project).
   // (coefficient snapshot: the diffusion law is evaluated by the kernel, and with tmass 2 the mass law
   // too -- the stored per-element value is then det J times the marker weight alone)
   const bool mass_in_kernel = layout_.tsnap && layout_.tmass == 2 && cmass_.gridfunc();
   CoeffDesc cm_one = cmass_;
   cm_one.kind = COEFF_CONSTANT;
   cm_one.value = 1.0;
   const double *cm_q = have_mass_ && !mass_in_kernel ? coeff_points(cmass_, ctmp_m_, s) : nullptr;
   const double *cd_q = have_diff_ && !layout_.tsnap ? coeff_points(cdiff_, ctmp_d_, s) : nullptr;

   const CoeffDesc *cm = have_mass_ ? (mass_in_kernel ? &cm_one : &cmass_) : nullptr;
   const CoeffDesc *cd = have_diff_ ? &cdiff_ : nullptr;
   if (layout_.affine())
   {
      kern::setup_affine(layout_, Q_, jac_ ? nullptr : enodes_.data(), jac_, W_.data(), cm, cd, cm_q, cd_q,
                         qd_diff_.data(), qd_mass_.data(), s);
      cdiag_ = false;
      if ((layout_.tsnap && layout_.kind == QLAYOUT_AFFINE) || layout_.kind == QLAYOUT_AFFINE_E)
      {
         if (cdflag_.size() < 1) { cdflag_.resize(1); }
         const char *e = std::getenv("ECM2_CDIAG");  // (A/B aid: 0 keeps the general flux product)
         cdiag_ = !(e && std::string(e) == "0") && kern::affine_c_diagonal(layout_, qd_diff_.data(), cdflag_.data(), s);
      }
   }
   else if (layout_.trilinear())
   {
      QPts qp = {};
      for (int q = 0; q < Q_ && q < MAX_Q1D; q++) { qp.x[q] = maps_.qpts[q]; }
      kern::setup_trilinear(layout_, Q_, jac_ ? nullptr : enodes_.data(), jac_ ? cfit_.data() : nullptr, W_.data(),
                            qp, cm, cd, cm_q, cd_q, qd_diff_.data(), qd_mass_.data(), s);
   }
   else if (jac_)
   {
      kern::setup_from_jacobians(layout_, jac_, W_.data(), cm, cd, cm_q, cd_q, qd_diff_.data(),
                                 qd_mass_.data(), s);
   }
   else
   {
      kern::setup_from_nodes(layout_, Q_, enodes_.data(), W_.data(), basis1_, cm, cd, cm_q, cd_q,
                             qd_diff_.data(), qd_mass_.data(), s);
   }
}

void PAForm::record_start(hipStream_t s)
{
   if (!timing_) { return; }
   if (ev_count_ >= ev_start_.size())
   {
      hipEvent_t a, b;
      ECM2_HIP(hipEventCreate(&a));
      ECM2_HIP(hipEventCreate(&b));
      ev_start_.push_back(a);
      ev_stop_.push_back(b);
   }
   ECM2_HIP(hipEventRecord(ev_start_[ev_count_], s));
}

void PAForm::record_stop(hipStream_t s)
{
   if (!timing_) { return; }
   ECM2_HIP(hipEventRecord(ev_stop_[ev_count_], s));
   ev_count_++;
}

void PAForm::timing_enable(bool on)
{
   timing_ = on;
   ev_count_ = 0;
}

void PAForm::timing_get(double *total_ms, long *launches)
{
   double t = 0.0;
   for (size_t i = 0; i < ev_count_; i++)
   {
      ECM2_HIP(hipEventSynchronize(ev_stop_[i]));
      float ms = 0.f;
      ECM2_HIP(hipEventElapsedTime(&ms, ev_start_[i], ev_stop_[i]));
      t += ms;
   }
   if (total_ms) { *total_ms = t; }
   if (launches) { *launches = (long)ev_count_; }
}

size_t PAForm::algorithmic_bytes() const
{
   // 8*NE*NQ*(6+1) qdata + 8*ndofs (x) + 8*ndofs (y) + 4*NE*ND (map).
   const size_t nc = (have_diff_ ? 6 : 0) + (have_mass_ ? 1 : 0);
   return 8ull * ne_ * NQ_ * nc + 16ull * n_owned_ + 4ull * ne_ * ND_;
}

void PAForm::ensure_csr()
{
   if (csr_off_.size() || ndofs_ == 0) { return; }
   // ElementRestriction ctor CSR build (restriction.cpp:68-106).
   std::vector<int> off(ndofs_ + 1, 0), idx((size_t)ne_ * ND_);
   for (int g : gmap_host_) { off[(g >= 0 ? g : -1 - g) + 1]++; }
   for (int i = 1; i <= ndofs_; i++) { off[i] += off[i - 1]; }
   for (size_t lid = 0; lid < gmap_host_.size(); lid++)
   {
      const int g = gmap_host_[lid];
      const int d = g >= 0 ? g : -1 - g;
      idx[off[d]++] = g >= 0 ? (int)lid : (int)(-1 - (long)lid);
   }
   for (int i = ndofs_; i > 0; i--) { off[i] = off[i - 1]; }
   off[0] = 0;
   csr_off_.upload(off);
   csr_idx_.upload(idx);
   ECM2_HIP(hipDeviceSynchronize());
}

void PAForm::ensure_work(hipStream_t)
{
   xe_.resize((size_t)ne_ * ND_);
   ye_.resize((size_t)ne_ * ND_);
}

void PAForm::mult(const double *x, double *y, hipStream_t s)
{
   ECM2_VERIFY(assembled_, ERR_STATE, "Mult before Assemble");
   ECM2_VERIFY(ndofs_ == 0 || (x && y), ERR_ARG, "null vector");
   if (ndofs_ == 0) { return; }
   const bool m = have_mass_, d = have_diff_;
   if (resolved_mode_ == KERNEL_UNFUSED)
   {
      // PABilinearFormExtension::MultInternal, bilinearform_ext.cpp:527-560.
      ensure_work(s);
      ensure_csr();
      record_start(s);
      kern::restriction_mult((long)ne_ * ND_, ND_, gmap_.data(), x, xe_.data(), s);
      if (ne_) { ECM2_HIP(hipMemsetAsync(ye_.data(), 0, ye_.bytes(), s)); }
      ApplyArgs a = apply_args(xe_.data(), nullptr, ye_.data(), nullptr, 0, layout_.nblk());
      if (m) { kern::apply_wpe(D_, Q_, true, false, a, true, true, basis_, s); }
      if (d) { kern::apply_wpe(D_, Q_, false, true, a, true, true, basis_, s); }
      kern::restriction_mult_transpose(ndofs_, ND_, csr_off_.data(), csr_idx_.data(), ye_.data(), y, s);
      record_stop(s);
      return;
   }
   if (!m && !d)
   {
      ECM2_HIP(hipMemsetAsync(y, 0, sizeof(double) * (size_t)ndofs_, s));
      return;
   }
   if (use_partials())
   {
      // exclusive dofs are plain-stored, shared ones summed from their partial slots:
      // every y entry is written exactly once, no memset, bitwise reproducible
      record_start(s);
      apply_blocks(x, nullptr, y, nullptr, 0, layout_.nblk(), s);
      record_stop(s);
      finish_shared(0, n_sh_, y, nullptr, s);
      return;
   }
   ECM2_HIP(hipMemsetAsync(y, 0, sizeof(double) * (size_t)ndofs_, s));
   record_start(s);
   apply_blocks(x, nullptr, y, nullptr, 0, layout_.nblk(), s);
   record_stop(s);
}

int PAForm::energy_parts() const
{
   // the coefficient-snapshot kernel (p = 2), one partial per 4-block workgroup.  (The p >= 3 brick kernel
   // folding the same sums was measured twice and rejected: every instantiation carrying the running sum
   // slowed the plain Mult by 3%; a separate instantiation cost the PCG's Mult what the dot pass it removed
   // cost -- profiles/r6/ab_brick_energy.txt.)
   const bool ts = assembled_ && use_partials() && resolved_mode_ == KERNEL_TPE && layout_.kind == QLAYOUT_AFFINE &&
                   layout_.tsnap && have_diff_ && D_ == 3 && Q_ == 4;
   return ts && ndofs_ > 0 ? (layout_.nblk() + 3) / 4 : 0;
}

void PAForm::mult_energy(const double *x, double *y, double *en, hipStream_t s)
{
   ECM2_VERIFY(energy_parts() > 0, ERR_UNSUPPORTED, "this form's Mult does not fold the energy");
   ECM2_VERIFY(x && y && en, ERR_ARG, "null vector");
   record_start(s);
   apply_blocks(x, nullptr, y, nullptr, 0, layout_.nblk(), s, false, en);
   record_stop(s);
   finish_shared(0, n_sh_, y, nullptr, s);
}

void PAForm::add_mult(const double *x, double *y, double a, hipStream_t s)
{
   ECM2_VERIFY(ndofs_ == 0 || y, ERR_ARG, "null vector");
   ywork_.resize(std::max(1, ndofs_));
   mult(x, ywork_.data(), s);
   kern::add_scaled(ndofs_, y, a, ywork_.data(), y, s);
}

void PAForm::set_scatter(int mode)
{
   ECM2_VERIFY(mode == SCATTER_PARTIALS || mode == SCATTER_ATOMIC, ERR_ARG, "unknown scatter mode " << mode);
   scatter_ = mode;
   gmap_line_.resize(0);  // the line kernel's bricks exist only with the partial scatter
   assembled_ = false;
}

void PAForm::finish_shared(int i0, int i1, double *y, double *yg, hipStream_t s)
{
   if (!use_partials()) { return; }
   // the plan's blocks cover the owned shared dofs [0, n_sh_owned_) then the ghost ones
   ECM2_VERIFY((i0 == 0 || i0 == n_sh_owned_) && (i1 == n_sh_owned_ || i1 == n_sh_) && i0 <= i1, ERR_INTERNAL,
               "summation range [" << i0 << ", " << i1 << ") is not a plan range");
   const int b0 = i0 == 0 ? 0 : sh_nblk_owned_, b1 = i1 == n_sh_owned_ ? sh_nblk_owned_ : sh_nblk_;
   kern::sum_partials(b0, b1, sh_blocks_.data(), sh_runs_.data(), sh_rslots_.data(), sh_pdof_.data(), part_.data(),
                      n_owned_, y, yg, s);
}

ApplyArgs PAForm::apply_args(const double *x, const double *xg, double *y, double *yg, int b0,
                             int b1) const
{
   ApplyArgs a;
   a.kind = layout_.kind;
   a.pw = layout_.pw;
   a.ne = ne_;
   a.blk_begin = b0;
   a.blk_end = b1;
   a.n_owned = n_owned_;
   a.pos = layout_.pos;
   a.lane_flags = lane_flags_.data();
   a.treg = treg_.size() ? treg_.data() : nullptr;
   a.treg_all = treg_all_ ? 1 : 0;
   a.tlat_all = tlat_all_ ? 1 : 0;
   a.lmap = lmap_.size() ? lmap_.data() : nullptr;
   for (int q = 0; q < Q_ && q < MAX_Q1D; q++) { a.qp.x[q] = maps_.qpts[q]; a.qw[q] = maps_.qw1[q]; }
   a.tsnap = layout_.tsnap ? tsnap_.data() : nullptr;
   a.tsnap_kind = layout_.tsnap;
   a.tmass = layout_.tmass;
   a.tlaw = layout_.tlaw;
   a.cdiag = cdiag_ && (layout_.tsnap || layout_.kind == QLAYOUT_AFFINE_E) ? 1 : 0;
   if (layout_.tsnap && layout_.tlaw)
   {
      a.law_d = point_law_of(cdiff_);
      if (layout_.tmass == 2 && cmass_.gridfunc()) { a.law_m = point_law_of(cmass_); }
   }
   a.xwave = (layout_.kind == QLAYOUT_AFFINE || layout_.kind == QLAYOUT_TRILINEAR) ? 1 : 0;
   a.part_stride = part_stride_;
   a.gmap = (resolved_mode_ == KERNEL_TPE) ? gmap_blk_.data()
            : (resolved_mode_ == KERNEL_LINE) ? gmap_line_.data() : gmap_.data();
   a.qdd = qd_diff_.data();
   a.qdm = qd_mass_.data();
   a.x = x; a.xg = xg; a.y = y; a.yg = yg;
   a.part = use_partials() ? const_cast<double *>(part_.data()) : nullptr;  // form-owned scratch
   a.btab = btab();
   a.lelem = lelem_.data();
   a.lelem_off = lelem_off_.empty() ? nullptr : lelem_off_.data();
   if (resolved_mode_ == KERNEL_LINE && use_partials())
   {
      a.part_brick = const_cast<double *>(part_.data());
      a.part = const_cast<double *>(part_.data()) + part_line_off_;  // leftovers: [e][nd] after the bricks
   }
   if (resolved_mode_ == KERNEL_LINE && brick_bz_)
   {
      a.brick_bz = brick_bz_;
      a.belem = belem_.data();
      a.bmap = bmap_.data();
      a.brick_off = brick_off_.data();
      a.breg = breg_.size() ? breg_.data() : nullptr;
   }
   return a;
}

void PAForm::apply_blocks(const double *x, const double *xg, double *y, double *yg, int b0, int b1,
                          hipStream_t s, bool latency, double *en)
{
   ECM2_VERIFY(assembled_, ERR_STATE, "apply before Assemble");
   ECM2_VERIFY(resolved_mode_ != KERNEL_UNFUSED, ERR_UNSUPPORTED, "block apply needs a fused kernel");
   if (resolved_mode_ == KERNEL_LINE && brick_bz_)
   {
      auto boundary = [&](int b) {
         return b == 0 || b == layout_.nblk() || std::find(splits_.begin(), splits_.end(), b) != splits_.end();
      };
      ECM2_VERIFY(boundary(b0) && boundary(b1), ERR_ARG, "apply_blocks [" << b0 << ", " << b1
                                                          << ") cuts a brick: declare the split with set_block_splits");
   }
   ApplyArgs a = apply_args(x, xg, y, yg, b0, b1);
   a.latency = latency && layout_.kind == QLAYOUT_AFFINE && have_mass_ && have_diff_ && !layout_.tsnap;
   a.en = en;  // (mult_energy: the snapshot kernel only)
   if (resolved_mode_ == KERNEL_TPE)
   {
      kern::apply_tpe(D_, Q_, have_mass_, have_diff_, a, basis_, rowtab_.data(), s);
   }
   else if (resolved_mode_ == KERNEL_LINE)
   {
      kern::apply_line(D_, Q_, have_mass_, have_diff_, a, s);
   }
   else
   {
      kern::apply_wpe(D_, Q_, have_mass_, have_diff_, a, false, false, basis_, s);
   }
}

void PAForm::assemble_diagonal(double *diag, hipStream_t s)
{
   ECM2_VERIFY(assembled_, ERR_STATE, "AssembleDiagonal before Assemble");
   if (ndofs_ == 0) { return; }
   // The diagonal is a function of the assembled state alone (every setter clears assembled_, and
   // Assemble bumps gen_): repeated requests between two Assembles -- a Jacobi smoother per PCG
   // solve, three SDIRK stages on one T -- copy the first result instead of recomputing it (at C4
   // with the snapshot: ~3 ms of expansion and diagonal kernels against a 25 us copy).
   if (diag_gen_ == gen_ && diag_cache_.size() == (size_t)ndofs_)
   {
      ECM2_HIP(hipMemcpyAsync(diag, diag_cache_.data(), diag_cache_.bytes(), hipMemcpyDeviceToDevice, s));
      return;
   }
   assemble_diagonal_uncached(diag, s);
   diag_cache_.resize(ndofs_);
   ECM2_HIP(hipMemcpyAsync(diag_cache_.data(), diag, diag_cache_.bytes(), hipMemcpyDeviceToDevice, s));
   diag_gen_ = gen_;
}

void PAForm::assemble_diagonal_uncached(double *diag, hipStream_t s)
{
   // The reference's AssembleDiagonal (bilinearform_ext.cpp:370-411) adds every integrator's
   // AssembleDiagonalPA into ONE localY and then zeroes a marked integrator's excluded elements of
   // that localY, so on those elements the contributions of the integrators added before it vanish
   // too (Mult masks each integrator's output separately, AddMultWithMarkers :753-774).  This
   // library reproduces it: when the second integrator added (S) is marked and excludes elements
   // the first (F) acts on, the diagonal is taken from a copy of the stored (Assemble-time) qdata
   // with F's entries multiplied by S's element weights (diag_w_, set at Assemble); the Mult's
   // qdata is swapped back whatever happens.
   if (diag_integ_ >= 0)
   {
      DeviceArray<double> td, tm;
      td.resize(qd_diff_.size());
      tm.resize(qd_mass_.size());
      if (td.size()) { ECM2_HIP(hipMemcpyAsync(td.data(), qd_diff_.data(), td.bytes(), hipMemcpyDeviceToDevice, s)); }
      if (tm.size()) { ECM2_HIP(hipMemcpyAsync(tm.data(), qd_mass_.data(), tm.bytes(), hipMemcpyDeviceToDevice, s)); }
      kern::scale_elements(layout_, diag_integ_, diag_w_.data(), td.data(), tm.data(), s);
      struct Swap
      {
         PAForm &f;
         DeviceArray<double> &d, &m;
         Swap(PAForm &f_, DeviceArray<double> &d_, DeviceArray<double> &m_) : f(f_), d(d_), m(m_)
         {
            std::swap(f.qd_diff_, d);
            std::swap(f.qd_mass_, m);
         }
         ~Swap()
         {
            (void)hipDeviceSynchronize();  // the temporaries are freed after this scope
            std::swap(f.qd_diff_, d);
            std::swap(f.qd_mass_, m);
         }
      } swap(*this, td, tm);
      diagonal_from_qdata(diag, s);
      return;
   }
   diagonal_from_qdata(diag, s);
}

void PAForm::diagonal_from_qdata(double *diag, hipStream_t s)
{
   if (resolved_mode_ == KERNEL_TPE && (have_mass_ || have_diff_))
   {
      // thread-per-element diagonal assembled like the Mult (deterministic with partials)
      double *dg = n_owned_ < ndofs_ ? diag + n_owned_ : nullptr;
      if (!use_partials()) { ECM2_HIP(hipMemsetAsync(diag, 0, sizeof(double) * (size_t)ndofs_, s)); }
      ApplyArgs a = apply_args(nullptr, nullptr, diag, dg, 0, layout_.nblk());
      DeviceArray<double> fd, fm;
      if (expand_needed())
      {
         expand_compressed(fd, fm, s);  // per-point qdata for the diagonal's tables
         a.kind = expand_kind();
         a.qdd = fd.data();
         a.qdm = fm.data();
      }
      kern::diagonal_tpe(D_, Q_, have_mass_, have_diff_, a, basis_, drowtab_.data(), s);
      finish_shared(0, n_sh_, diag, dg, s);
      if (fd.size()) { ECM2_HIP(hipStreamSynchronize(s)); }  // the temporaries are freed on return
      return;
   }
   ECM2_HIP(hipMemsetAsync(diag, 0, sizeof(double) * (size_t)ndofs_, s));
   DeviceArray<double> fd, fm;
   int kind = layout_.kind;
   const double *qdd = qd_diff_.data(), *qdm = qd_mass_.data();
   if (expand_needed())
   {
      expand_compressed(fd, fm, s);
      kind = expand_kind();
      qdd = fd.data();
      qdm = fm.data();
   }
   kern::diagonal(layout_.pos, D_, Q_, kind, ne_, gmap_.data(), have_diff_ ? qdd : nullptr,
                  have_mass_ ? qdm : nullptr, diag, false, basis_, btab(), s);
   if (fd.size()) { ECM2_HIP(hipStreamSynchronize(s)); }  // the temporaries are freed on return
}

void PAForm::expand_compressed(DeviceArray<double> &fd, DeviceArray<double> &fm, hipStream_t s) const
{
   QLayout L = layout_;
   L.kind = expand_kind();
   fd.resize(std::max<size_t>(1, have_diff_ ? L.diff_size() : 0));
   fm.resize(std::max<size_t>(1, have_mass_ ? L.mass_size() : 0));
   if (L.blocked() && ne_ % kElemBlock)
   {
      ECM2_HIP(hipMemsetAsync(fd.data(), 0, fd.bytes(), s));
      ECM2_HIP(hipMemsetAsync(fm.data(), 0, fm.bytes(), s));
   }
   QPts qp = {};
   for (int q = 0; q < Q_ && q < MAX_Q1D; q++) { qp.x[q] = maps_.qpts[q]; }
   if (layout_.tsnap)
   {
      // beta (and a mass law of the same field) at the points from the snapshot -- the field as
      // Assemble saw it, projected as the reference's setup projects a GridFunctionCoefficient and the
      // law applied at the point -- times the STORED element matrices and mass values (which the
      // marker diagonal may have scaled, assemble_diagonal)
      DeviceArray<double> tdof, ctd, ctm;
      const double *tv = tsnap_.data();
      if (layout_.tsnap == 2)
      {
         tdof.resize(std::max(1, ndofs_));
         kern::lattice_to_dofs(layout_.nblk(), tpe_lattice_points(D_), lmap_.data(), tsnap_.data(), tdof.data(), s);
         tv = tdof.data();
      }
      CoeffDesc cs = cdiff_;
      cs.kind = layout_.tlaw ? cdiff_.kind : COEFF_GRIDFUNC;  // (tlaw 0: the law is in the snapshot)
      cs.lvec = tv;
      cs.emask = nullptr;
      const double *cd_q = coeff_points(cs, ctd, s);
      const double *cm_q = nullptr;
      if (layout_.tmass == 2 && cmass_.gridfunc())
      {
         CoeffDesc cm = cmass_;
         cm.lvec = tv;  // tlaw 1: the snapshot is the field itself
         cm.emask = nullptr;
         cm_q = coeff_points(cm, ctm, s);
      }
      kern::tsnap_expand(layout_, Q_, W_.data(), qd_diff_.data(), qd_mass_.data(), cd_q, cm_q, fd.data(),
                         fm.data(), s);
      ECM2_HIP(hipStreamSynchronize(s));  // the temporaries are freed on return
      return;
   }
   if (layout_.trilinear())
   {
      kern::trilinear_expand(layout_, Q_, qd_diff_.data(), qd_mass_.data(), qp, fd.data(), fm.data(), s);
   }
   else { kern::affine_expand(layout_, Q_, qd_diff_.data(), qd_mass_.data(), fd.data(), fm.data(), s); }
}

void PAForm::restriction_mult(const double *x, double *xe, hipStream_t s)
{
   kern::restriction_mult((long)ne_ * ND_, ND_, gmap_.data(), x, xe, s);
}

void PAForm::restriction_mult_transpose(const double *xe, double *y, hipStream_t s)
{
   ensure_csr();
   kern::restriction_mult_transpose(ndofs_, ND_, csr_off_.data(), csr_idx_.data(), xe, y, s);
}

void PAForm::integrator_add_mult(int kind, const double *xe, double *ye, hipStream_t s)
{
   ECM2_VERIFY(assembled_, ERR_STATE, "AddMultPA before Assemble");
   ECM2_VERIFY((kind == INTEG_MASS && have_mass_) || (kind == INTEG_DIFFUSION && have_diff_),
               ERR_ARG, "integrator " << kind << " not present");
   ApplyArgs a = apply_args(xe, nullptr, ye, nullptr, 0, layout_.nblk());
   a.gmap = gmap_.data();
   DeviceArray<double> fd, fm;
   if (expand_needed())
   {
      expand_compressed(fd, fm, s);
      a.kind = expand_kind();
      a.qdd = fd.data();
      a.qdm = fm.data();
   }
   kern::apply_wpe(D_, Q_, kind == INTEG_MASS, kind == INTEG_DIFFUSION, a, true, true, basis_, s);
   if (fd.size()) { ECM2_HIP(hipStreamSynchronize(s)); }
}

void PAForm::get_qdata(int kind, double *out, hipStream_t s)
{
   ECM2_VERIFY(assembled_, ERR_STATE, "get_qdata before Assemble");
   const bool diff = kind == INTEG_DIFFUSION;
   ECM2_VERIFY(diff ? have_diff_ : have_mass_, ERR_ARG, "integrator " << kind << " not present");
   DeviceArray<double> fd, fm;
   const bool tl = expand_needed();  // TRILINEAR(_E), or a diffusion-only AFFINE(_E) form
   const bool aff = layout_.affine() && !tl;
   if (tl) { expand_compressed(fd, fm, s); }  // decoded as expand_kind() below
   const int kind_h = tl ? expand_kind() : layout_.kind;
   DeviceArray<double> &src = tl ? (diff ? fd : fm) : ((diff && !aff) ? qd_diff_ : qd_mass_);
   std::vector<double> h(src.size()), hc(aff ? qd_diff_.size() : 0);
   if (src.size())
   {
      ECM2_HIP(hipMemcpyAsync(h.data(), src.data(), src.bytes(), hipMemcpyDeviceToHost, s));
   }
   if (hc.size())
   {
      ECM2_HIP(hipMemcpyAsync(hc.data(), qd_diff_.data(), qd_diff_.bytes(), hipMemcpyDeviceToHost, s));
   }
   ECM2_HIP(hipStreamSynchronize(s));
   const int nc = diff ? (layout_.kind == QLAYOUT_NATIVE9 ? 9 : 6) : 1;
   std::vector<int> invp;
   if (!perm_host_.empty())
   {
      invp.resize(ne_);
      for (int i = 0; i < ne_; i++) { invp[perm_host_[i]] = i; }
   }
   auto inv_perm = [&](int e) { return invp[e]; };
   for (int e = 0; e < ne_; e++)
      for (int c = 0; c < nc; c++)
         for (int q = 0; q < NQ_; q++)
         {
            size_t src_i;
            if (kind_h == QLAYOUT_NATIVE || kind_h == QLAYOUT_NATIVE9) { src_i = ((size_t)e * nc + c) * NQ_ + q; }
            else if (kind_h == QLAYOUT_AFFINE_E)
            {
               const size_t pi = ((size_t)e * NQ_ + q) * 2;
               out[((size_t)e * nc + c) * NQ_ + q] = diff ? h[pi] * hc[(size_t)e * 6 + c] : h[pi + 1];
               continue;
            }
            else
            {
               const int ip = perm_host_.empty() ? e : inv_perm(e);
               const int blk = ip / 64, lane = ip % 64;
               if (aff)
               {
                  // AFFINE: D_c(q) = (W beta)(q) * C_c, mass = the pair's second entry
                  const size_t pi = (((size_t)blk * NQ_ + q) * 64 + lane) * 2;
                  out[((size_t)e * nc + c) * NQ_ + q] =
                     diff ? h[pi] * hc[(((size_t)blk * 3 + c / 2) * 64 + lane) * 2 + (c & 1)] : h[pi + 1];
                  continue;
               }
               if (diff) { src_i = (((size_t)blk * NQ_ + q) * 3 + c / 2) * 128 + lane * 2 + (c & 1); }
               else { src_i = ((size_t)blk * ((NQ_ + 1) / 2) + q / 2) * 128 + lane * 2 + (q & 1); }
            }
            out[((size_t)e * nc + c) * NQ_ + q] = h[src_i];
         }
}

// --------------------------------------------------------------------------
// Device PCG
// --------------------------------------------------------------------------

} // namespace ecm2
