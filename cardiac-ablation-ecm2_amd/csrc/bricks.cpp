// bricks.cpp -- see bricks.hpp.
#include "bricks.hpp"

#include <algorithm>
#include <cstdint>
#include <deque>
#include <unordered_map>

namespace ecm2
{

namespace
{
inline int dof_of(int g) { return g >= 0 ? g : -1 - g; }

// local index of the (i, j) entry of the face of direction dir at level s (0 or D-1)
inline int face_entry(int D, int dir, int s, int i, int j)
{
   if (dir == 0) { return (j * D + i) * D + s; }
   if (dir == 1) { return (j * D + s) * D + i; }
   return (s * D + j) * D + i;
}
} // namespace

FaceNeighbors face_neighbors(int ne, int D, const std::vector<int> &gm)
{
   const int ND = D * D * D;
   auto dof = [&](int e, int a) { return dof_of(gm[(size_t)e * ND + a]); };
   auto key = [&](int e, int dir, int s) {
      uint64_t h = 1469598103934665603ull;  // FNV-1a over the face's four corner dofs
      for (int j : {0, D - 1})
         for (int i : {0, D - 1}) { h = (h ^ (uint64_t)(uint32_t)dof(e, face_entry(D, dir, s, i, j))) * 1099511628211ull; }
      return h;
   };
   FaceNeighbors N;
   for (int dir = 0; dir < 3; dir++)
   {
      N.n[dir].assign(ne, -1);
      std::unordered_map<uint64_t, int> low;
      low.reserve((size_t)ne * 2);
      for (int e = 0; e < ne; e++)
      {
         auto it = low.emplace(key(e, dir, 0), e);
         if (!it.second) { it.first->second = -1; }  // ambiguous: no link through it
      }
      for (int e = 0; e < ne; e++)
      {
         auto it = low.find(key(e, dir, D - 1));
         if (it == low.end() || it->second < 0 || it->second == e) { continue; }
         const int f = it->second;
         bool ok = true;
         for (int j = 0; j < D && ok; j++)
            for (int i = 0; i < D && ok; i++)
            {
               ok = dof(e, face_entry(D, dir, D - 1, i, j)) == dof(f, face_entry(D, dir, 0, i, j));
            }
         if (ok) { N.n[dir][e] = f; }
      }
   }
   return N;
}

std::vector<int> face_brick_order(int ne, int D, const std::vector<int> &gm)
{
   std::vector<int> perm;
   perm.reserve(ne);
   if (ne == 0) { return perm; }
   const FaceNeighbors N = face_neighbors(ne, D, gm);
   std::vector<int> lo[3];
   for (int d = 0; d < 3; d++)
   {
      lo[d].assign(ne, -1);
      for (int e = 0; e < ne; e++) { if (N.n[d][e] >= 0) { lo[d][N.n[d][e]] = e; } }
   }
   // lattice coordinates per connected patch (breadth-first over the links)
   std::vector<int> patch(ne, -1), c[3];
   for (int d = 0; d < 3; d++) { c[d].assign(ne, 0); }
   std::vector<int> pmin;  // per patch: min coordinate (3 per patch)
   std::deque<int> q;
   int np = 0;
   for (int e0 = 0; e0 < ne; e0++)
   {
      if (patch[e0] >= 0) { continue; }
      patch[e0] = np;
      int mn[3] = {0, 0, 0};
      q.push_back(e0);
      while (!q.empty())
      {
         const int e = q.front();
         q.pop_front();
         for (int d = 0; d < 3; d++)
         {
            mn[d] = std::min(mn[d], c[d][e]);
            for (int s : {1, -1})
            {
               const int f = s > 0 ? N.n[d][e] : lo[d][e];
               if (f < 0 || patch[f] >= 0) { continue; }
               patch[f] = np;
               for (int k = 0; k < 3; k++) { c[k][f] = c[k][e] + (k == d ? s : 0); }
               q.push_back(f);
            }
         }
      }
      pmin.insert(pmin.end(), mn, mn + 3);
      np++;
   }
   // group by (patch, 4-aligned cell); a group is a brick when it has all 64 positions
   // and every internal link
   auto cell = [&](int e) -> uint64_t {
      const int p = patch[e];
      uint64_t k = (uint64_t)p;
      for (int d = 0; d < 3; d++) { k = k << 14 | (uint64_t)((c[d][e] - pmin[3 * p + d]) / 4); }
      return k;
   };
   auto local = [&](int e) {
      const int p = patch[e];
      int l = 0;
      for (int d = 2; d >= 0; d--) { l = l * 4 + (c[d][e] - pmin[3 * p + d]) % 4; }
      return l;  // ax + 4 ay + 16 az
   };
   std::unordered_map<uint64_t, std::vector<int>> groups;
   groups.reserve((size_t)ne / 32 + 1);
   bool coords_fit = true;
   for (int e = 0; e < ne; e++)
   {
      for (int d = 0; d < 3; d++) { coords_fit &= (c[d][e] - pmin[3 * patch[e] + d]) < (1 << 16); }
   }
   if (coords_fit && np < (1 << 20))
   {
      for (int e = 0; e < ne; e++) { groups[cell(e)].push_back(e); }
   }
   // bricks along a Morton curve of their cells within each patch (patches in order of
   // their first element): neighbouring bricks, which gather the same x values, run close
   // in time (x-gather L2 locality)
   auto spread = [](uint64_t v) {
      v &= 0x1fffff;
      v = (v | v << 32) & 0x1f00000000ffffull;
      v = (v | v << 16) & 0x1f0000ff0000ffull;
      v = (v | v << 8) & 0x100f00f00f00f00full;
      v = (v | v << 4) & 0x10c30c30c30c30c3ull;
      v = (v | v << 2) & 0x1249249249249249ull;
      return v;
   };
   auto curve = [&](int e) -> uint64_t {
      const int p = patch[e];
      uint64_t m = 0;
      for (int d = 0; d < 3; d++) { m |= spread((uint64_t)((c[d][e] - pmin[3 * p + d]) / 4)) << d; }
      return m;
   };
   std::vector<std::pair<std::pair<int, uint64_t>, std::vector<int>>> bricks;  // ((patch, curve), lanes)
   std::vector<char> used(ne, 0);
   for (auto &kv : groups)
   {
      const std::vector<int> &g = kv.second;
      if (g.size() != 64) { continue; }
      std::vector<int> lane(64, -1);
      bool ok = true;
      for (int e : g)
      {
         int &s = lane[local(e)];
         ok &= s < 0;
         s = e;
      }
      for (int l = 0; l < 64 && ok; l++)
      {
         const int a[3] = {l % 4, (l / 4) % 4, l / 16}, step[3] = {1, 4, 16};
         for (int d = 0; d < 3 && ok; d++) { ok = a[d] == 3 || N.n[d][lane[l]] == lane[l + step[d]]; }
      }
      if (!ok) { continue; }
      // (bricks in the caller's element order -- the reference's space-filling curve on its own
      // meshes -- measured 1.3% slower at C4 with the reference's numbering, equal at C3:
      // profiles/r3_ab_order.txt)
      bricks.push_back({{patch[lane[0]], curve(lane[0])}, lane});
   }
   std::sort(bricks.begin(), bricks.end(), [](const auto &a, const auto &b) { return a.first < b.first; });
   for (auto &b : bricks)
   {
      for (int e : b.second)
      {
         perm.push_back(e);
         used[e] = 1;
      }
   }
   for (int e = 0; e < ne; e++) { if (!used[e]) { perm.push_back(e); } }
   return perm;
}

void find_bricks(int ne, int D, const std::vector<int> &gm, int bz, const std::vector<int> &seg,
                 std::vector<int> &belem, std::vector<char> &in_brick)
{
   const int ND = D * D * D;
   const FaceNeighbors nb = face_neighbors(ne, D, gm);
   const int nbe = 4 * bz;
   for (int e0 = 0; e0 < ne; e0++)
   {
      if (in_brick[e0]) { continue; }
      std::vector<int> el(nbe, -1);
      el[0] = e0;
      el[1] = nb(0, e0);
      el[2] = nb(1, e0);
      el[3] = nb(0, el[2]);
      bool ok = el[1] >= 0 && el[3] >= 0 && nb(1, el[1]) == el[3];
      // further 2 x 2 layers (bz = 2; column bricks bz = 4, 8): linked in z to the layer
      // below and in x / y among themselves
      for (int z = 1; z < bz && ok; z++)
      {
         int *l = el.data() + 4 * z;
         for (int i = 0; i < 4; i++) { l[i] = nb(2, l[i - 4]); }
         ok = l[0] >= 0 && l[1] >= 0 && l[2] >= 0 && l[3] >= 0 && nb(0, l[0]) == l[1] &&
              nb(1, l[0]) == l[2] && nb(0, l[2]) == l[3] && nb(1, l[1]) == l[3];
      }
      for (int i = 0; i < nbe && ok; i++)
      {
         ok = el[i] >= 0 && !in_brick[el[i]] && seg[el[i]] == seg[e0];
         for (int j = 0; j < i && ok; j++) { ok = el[j] != el[i]; }
         for (int a = 0; a < ND && ok; a++) { ok = gm[(size_t)el[i] * ND + a] >= 0; }
      }
      if (!ok) { continue; }
      for (int i = 0; i < nbe; i++)
      {
         belem.push_back(el[i]);
         in_brick[el[i]] = 1;
      }
   }
}

} // namespace ecm2
