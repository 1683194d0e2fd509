// partition.cpp -- see partition.hpp.
#include "partition.hpp"
#include "common.hpp"

#include <algorithm>
#include <cstdint>

namespace ecm2
{

std::vector<int> partition_slabs_z(const HexMesh &m, int nranks)
{
   ECM2_VERIFY(m.nx > 0, ERR_ARG, "slab partition needs a Cartesian mesh");
   ECM2_VERIFY(nranks >= 1 && nranks <= m.nz, ERR_ARG, "bad rank count " << nranks);
   std::vector<int> er(m.ne);
   for (int e = 0; e < m.ne; e++)
   {
      const long ez = m.lex_index(e) / (m.nx * m.ny);
      // Mesh::CartesianPartitioning (mesh.cpp:8994) with nxyz = (1, 1, R) on the element centre
      // z = (ez + 1/2) / nz of the box: r = floor(R (ez + 1/2) / nz), in exact integer arithmetic
      er[e] = (int)std::min<long>(nranks - 1, (2 * ez + 1) * nranks / (2L * m.nz));
   }
   return er;
}

std::vector<int> partition_bricks(const HexMesh &m, int nranks, int cell)
{
   ECM2_VERIFY(m.nx > 0, ERR_ARG, "brick partition needs a Cartesian mesh");
   ECM2_VERIFY(cell >= 1, ERR_ARG, "bad brick edge " << cell);
   const long bx = (m.nx + cell - 1) / cell, by = (m.ny + cell - 1) / cell, bz = (m.nz + cell - 1) / cell;
   const long nb = bx * by * bz;
   ECM2_VERIFY(nranks >= 1 && nranks <= nb, ERR_ARG, "bad rank count " << nranks << " for " << nb << " bricks");
   std::vector<int> er(m.ne);
   for (int e = 0; e < m.ne; e++)
   {
      const long l = m.lex_index(e), ix = l % m.nx, iy = (l / m.nx) % m.ny, iz = l / ((long)m.nx * m.ny);
      const long b = ix / cell + bx * (iy / cell + by * (iz / cell));
      er[e] = (int)(b * nranks / nb);  // equal runs of the lexicographic brick order
   }
   return er;
}

LocalPart build_local_part(const H1Space &s, const std::vector<int> &elem_rank, int rank, int nranks,
                           const HexMesh *cart, bool overlap)
{
   ECM2_VERIFY((int)elem_rank.size() == s.ne, ERR_ARG, "elem_rank size " << elem_rank.size() << " != ne " << s.ne);
   ECM2_VERIFY(nranks >= 1 && nranks <= 64, ERR_UNSUPPORTED, "1..64 ranks supported");
   ECM2_VERIFY(rank >= 0 && rank < nranks, ERR_ARG, "bad rank " << rank);
   LocalPart p;
   p.rank = rank;
   p.nranks = nranks;
   p.overlap = overlap;
   p.order = s.order;
   p.nd = s.nd;
   const int nd = s.nd;
   // which ranks touch each dof
   std::vector<uint64_t> touch(s.ndofs, 0);
   for (int e = 0; e < s.ne; e++)
   {
      const int r = elem_rank[e];
      ECM2_VERIFY(r >= 0 && r < nranks, ERR_ARG, "element rank " << r << " out of range");
      for (int a = 0; a < nd; a++)
      {
         const int g = s.gather_map[(size_t)e * nd + a];
         touch[g >= 0 ? g : -1 - g] |= (1ull << r);
      }
   }
   auto owner = [&](int g) { return __builtin_ctzll(touch[g]); };
   const uint64_t me = 1ull << rank;
   auto dofg = [](int g) { return g >= 0 ? g : -1 - g; };
   // local elements of each rank: owned ones, plus (OVERLAP) every element touching a dof the
   // rank owns; need[g] = ranks whose local elements touch dof g
   auto is_local = [&](int e, int r) {
      if (elem_rank[e] == r) { return true; }
      if (!overlap) { return false; }
      for (int a = 0; a < nd; a++) { if (owner(dofg(s.gather_map[(size_t)e * nd + a])) == r) { return true; } }
      return false;
   };
   std::vector<uint64_t> need(touch);
   if (overlap)
   {
      for (int e = 0; e < s.ne; e++)
      {
         uint64_t ranks = 0;  // owners of e's dofs: e is local to each of them
         for (int a = 0; a < nd; a++) { ranks |= 1ull << owner(dofg(s.gather_map[(size_t)e * nd + a])); }
         for (int a = 0; a < nd; a++) { need[dofg(s.gather_map[(size_t)e * nd + a])] |= ranks; }
      }
   }
   // local dofs
   std::vector<int> owned, ghost;
   for (int g = 0; g < s.ndofs; g++)
   {
      if (!(need[g] & me)) { continue; }
      if (owner(g) == rank) { owned.push_back(g); }
      else { ghost.push_back(g); }
   }
   std::stable_sort(ghost.begin(), ghost.end(), [&](int a, int b) { return owner(a) < owner(b); });
   p.n_owned = (int)owned.size();
   p.n_ghost = (int)ghost.size();
   p.local_to_global = owned;
   p.local_to_global.insert(p.local_to_global.end(), ghost.begin(), ghost.end());
   std::vector<int> g2l(s.ndofs, -1);
   for (int i = 0; i < (int)p.local_to_global.size(); i++) { g2l[p.local_to_global[i]] = i; }
   // neighbours: ranks that own my ghosts or ghost my owned dofs
   uint64_t nb = 0;
   for (int g : owned) { nb |= need[g] & ~me; }
   for (int g : ghost) { nb |= 1ull << owner(g); }
   for (int r = 0; r < nranks; r++) { if (nb & (1ull << r)) { p.nbrs.push_back(r); } }
   p.send_off.assign(1, 0);
   p.recv_off.assign(1, 0);
   for (int r : p.nbrs)
   {
      for (int i = 0; i < p.n_owned; i++)
      {
         if (need[owned[i]] & (1ull << r)) { p.send_idx.push_back(i); }
      }
      p.send_off.push_back((int)p.send_idx.size());
      int cnt = 0;
      for (int g : ghost) { cnt += owner(g) == r; }
      p.recv_off.push_back(p.recv_off.back() + cnt);
   }
   // local elements: interior (no ghost dof) first, then boundary
   std::vector<int> interior, boundary;
   for (int e = 0; e < s.ne; e++)
   {
      if (!is_local(e, rank)) { continue; }
      p.ne_owned += elem_rank[e] == rank;
      bool bnd = false;
      for (int a = 0; a < nd && !bnd; a++)
      {
         const int g = s.gather_map[(size_t)e * nd + a];
         bnd = g2l[g >= 0 ? g : -1 - g] >= p.n_owned;
      }
      (bnd ? boundary : interior).push_back(e);
   }
   if (cart && cart->nx > 0)
   {
      interior = brick_order(interior, *cart);
      boundary = brick_order(boundary, *cart);
   }
   p.ne_interior = (int)interior.size();
   p.elems = interior;
   p.elems.insert(p.elems.end(), boundary.begin(), boundary.end());
   p.ne_local = (int)p.elems.size();
   p.gather_map.resize((size_t)p.ne_local * nd);
   for (int le = 0; le < p.ne_local; le++)
   {
      const int e = p.elems[le];
      for (int a = 0; a < nd; a++)
      {
         const int g = s.gather_map[(size_t)e * nd + a];
         const int l = g2l[g >= 0 ? g : -1 - g];
         p.gather_map[(size_t)le * nd + a] = g >= 0 ? l : -1 - l;
      }
   }
   return p;
}

std::vector<Xfer> exchange_schedule(const LocalPart &p, bool transpose)
{
   std::vector<Xfer> out;
   for (size_t k = 0; k < p.nbrs.size(); k++)
   {
      const int s0 = p.send_off[k], s1 = p.send_off[k + 1];  // my owned dofs neighbour k ghosts
      const int r0 = p.recv_off[k], r1 = p.recv_off[k + 1];  // my ghosts owned by neighbour k
      const int nb = p.nbrs[k];
      if (!transpose)
      {
         if (s1 > s0)
         {
            bool contig = true;
            for (int i = s0 + 1; i < s1 && contig; i++) { contig = p.send_idx[i] == p.send_idx[i - 1] + 1; }
            out.push_back(contig ? Xfer{nb, 1, XBUF_X_TRUE, p.send_idx[s0], s1 - s0}
                                 : Xfer{nb, 1, XBUF_SENDBUF, s0, s1 - s0});
         }
         if (r1 > r0) { out.push_back(Xfer{nb, 0, XBUF_XGHOST, r0, r1 - r0}); }
      }
      else
      {
         if (r1 > r0) { out.push_back(Xfer{nb, 1, XBUF_YGHOST, r0, r1 - r0}); }
         if (s1 > s0) { out.push_back(Xfer{nb, 0, XBUF_RECVBUF, s0, s1 - s0}); }
      }
   }
   return out;
}

} // namespace ecm2
