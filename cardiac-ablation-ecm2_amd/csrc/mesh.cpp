// mesh.cpp -- see mesh.hpp for reference citations.
#include "mesh.hpp"
#include "common.hpp"
#include "fe.hpp"

#include <algorithm>
#include <string>
#include <cstdlib>
#include <array>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <unordered_map>

namespace ecm2
{

const int kLexToNative[8] = {0, 1, 3, 2, 4, 5, 7, 6};

HexMesh HexMesh::cartesian(int nx, int ny, int nz, double sx, double sy, double sz)
{
   ECM2_VERIFY(nx > 0 && ny > 0 && nz > 0, ERR_ARG, "bad Cartesian size");
   HexMesh m;
   m.nx = nx; m.ny = ny; m.nz = nz;
   m.nv = (nx + 1) * (ny + 1) * (nz + 1);
   m.ne = nx * ny * nz;
   m.vert.resize((size_t)m.nv * 3);
   size_t v = 0;
   for (int z = 0; z <= nz; z++)
      for (int y = 0; y <= ny; y++)
         for (int x = 0; x <= nx; x++, v++)
         {
            m.vert[3 * v + 0] = ((double)x / nx) * sx;
            m.vert[3 * v + 1] = ((double)y / ny) * sy;
            m.vert[3 * v + 2] = ((double)z / nz) * sz;
         }
   auto vtx = [&](int x, int y, int z) { return x + (y + z * (ny + 1)) * (nx + 1); };
   m.elem.resize((size_t)m.ne * 8);
   m.attr.assign(m.ne, 1);
   size_t e = 0;
   // Lexicographic element order (Make3D without sfc_ordering).
   for (int z = 0; z < nz; z++)
      for (int y = 0; y < ny; y++)
         for (int x = 0; x < nx; x++, e++)
         {
            int *ind = &m.elem[8 * e];
            ind[0] = vtx(x, y, z);     ind[1] = vtx(x + 1, y, z);
            ind[2] = vtx(x + 1, y + 1, z); ind[3] = vtx(x, y + 1, z);
            ind[4] = vtx(x, y, z + 1); ind[5] = vtx(x + 1, y, z + 1);
            ind[6] = vtx(x + 1, y + 1, z + 1); ind[7] = vtx(x, y + 1, z + 1);
         }
   return m;
}

namespace
{
bool next_content_line(std::istream &in, std::string &line)
{
   while (std::getline(in, line))
   {
      const size_t h = line.find('#');
      if (h != std::string::npos) { line.erase(h); }
      const size_t b = line.find_first_not_of(" \t\r");
      if (b == std::string::npos) { continue; }
      line = line.substr(b);
      while (!line.empty() && (line.back() == ' ' || line.back() == '\r' || line.back() == '\t'))
      {
         line.pop_back();
      }
      if (!line.empty()) { return true; }
   }
   return false;
}
} // namespace

HexMesh HexMesh::read(const std::string &path)
{
   std::ifstream in(path);
   ECM2_VERIFY(in.good(), ERR_IO, "cannot open mesh file '" << path << "'");
   std::string line;
   ECM2_VERIFY(next_content_line(in, line), ERR_IO, "empty mesh file");
   if (line.rfind("MFEM INLINE mesh v1.0", 0) == 0)
   {
      // mesh_readers.cpp:1356-1506: key = value pairs; only hex is supported here.
      std::string type;
      int nx = 0, ny = 0, nz = 0;
      double sx = 1.0, sy = 1.0, sz = 1.0;
      while (next_content_line(in, line))
      {
         const size_t eq = line.find('=');
         if (eq == std::string::npos) { continue; }
         std::string key = line.substr(0, eq), val = line.substr(eq + 1);
         key.erase(key.find_last_not_of(" \t") + 1);
         val.erase(0, val.find_first_not_of(" \t"));
         if (key == "type") { type = val; }
         else if (key == "nx") { nx = std::stoi(val); }
         else if (key == "ny") { ny = std::stoi(val); }
         else if (key == "nz") { nz = std::stoi(val); }
         else if (key == "sx") { sx = std::stod(val); }
         else if (key == "sy") { sy = std::stod(val); }
         else if (key == "sz") { sz = std::stod(val); }
      }
      ECM2_VERIFY(type == "hex" || type == "hexahedron", ERR_UNSUPPORTED,
                  "INLINE mesh type '" << type << "' not supported (hex only)");
      return cartesian(nx, ny, nz, sx, sy, sz);
   }
   ECM2_VERIFY(line.rfind("MFEM mesh v1.0", 0) == 0, ERR_IO,
               "unsupported mesh format header '" << line << "'");
   HexMesh m;
   int dim = 0;
   while (next_content_line(in, line))
   {
      if (line == "dimension")
      {
         next_content_line(in, line);
         dim = std::stoi(line);
         ECM2_VERIFY(dim == 3, ERR_UNSUPPORTED, "only 3D meshes are supported");
      }
      else if (line == "elements")
      {
         next_content_line(in, line);
         m.ne = std::stoi(line);
         m.elem.resize((size_t)m.ne * 8);
         m.attr.resize(m.ne);
         for (int e = 0; e < m.ne; e++)
         {
            ECM2_VERIFY(next_content_line(in, line), ERR_IO, "truncated elements");
            std::istringstream ls(line);
            int a, g;
            ls >> a >> g;
            ECM2_VERIFY(g == 5, ERR_UNSUPPORTED, "element geometry " << g << " (only hex = 5)");
            m.attr[e] = a;
            for (int k = 0; k < 8; k++) { ls >> m.elem[8 * e + k]; }
         }
      }
      else if (line == "boundary")
      {
         // The boundary is re-derived from the element faces (conforming meshes).
         next_content_line(in, line);
         const int nb = std::stoi(line);
         for (int b = 0; b < nb; b++) { next_content_line(in, line); }
      }
      else if (line == "vertices")
      {
         next_content_line(in, line);
         m.nv = std::stoi(line);
         next_content_line(in, line);
         const int sdim = std::stoi(line);
         ECM2_VERIFY(sdim == 3, ERR_UNSUPPORTED, "vertex dimension " << sdim);
         m.vert.resize((size_t)m.nv * 3);
         for (int v = 0; v < m.nv; v++)
         {
            ECM2_VERIFY(next_content_line(in, line), ERR_IO, "truncated vertices");
            std::istringstream ls(line);
            ls >> m.vert[3 * v] >> m.vert[3 * v + 1] >> m.vert[3 * v + 2];
         }
      }
      else if (line == "nodes")
      {
         ECM2_VERIFY(false, ERR_UNSUPPORTED, "curved (nodal) meshes are not supported");
      }
   }
   ECM2_VERIFY(m.ne > 0 && m.nv > 0, ERR_IO, "mesh has no elements or vertices");
   for (int v : m.elem) { ECM2_VERIFY(v >= 0 && v < m.nv, ERR_IO, "vertex index out of range"); }
   return m;
}

void HexMesh::refine_uniform()
{
   // Each hex -> 8 children on the parent's 3x3x3 lattice; new vertices are the
   // edge midpoints, face centres and element centre (averages of the parent's
   // corners = the trilinear map at 1/2), shared through edge/face keys.
   std::vector<double> nvert(vert);
   std::map<std::pair<int, int>, int> edge_mid;
   std::map<std::array<int, 4>, int> face_mid;
   auto add_vertex = [&](const double *p) {
      nvert.push_back(p[0]); nvert.push_back(p[1]); nvert.push_back(p[2]);
      return (int)(nvert.size() / 3 - 1);
   };
   std::vector<int> nelem;
   nelem.reserve((size_t)ne * 64);
   std::vector<int> nattr;
   nattr.reserve((size_t)ne * 8);
   for (int e = 0; e < ne; e++)
   {
      int corner[8];  // lexicographic
      for (int a = 0; a < 8; a++) { corner[a] = elem[8 * e + kLexToNative[a]]; }
      int lat[27];    // lattice (I,J,K) in {0,1,2}^3 -> vertex id
      for (int K = 0; K < 3; K++)
         for (int J = 0; J < 3; J++)
            for (int I = 0; I < 3; I++)
            {
               // corners of the lattice point's parent entity
               int lo[3] = {I == 2, J == 2, K == 2}, hi[3] = {I != 0, J != 0, K != 0};
               std::vector<int> ids;
               double p[3] = {0, 0, 0};
               for (int cz = lo[2]; cz <= hi[2]; cz++)
                  for (int cy = lo[1]; cy <= hi[1]; cy++)
                     for (int cx = lo[0]; cx <= hi[0]; cx++)
                     {
                        const int v = corner[cx + 2 * cy + 4 * cz];
                        ids.push_back(v);
                        for (int c = 0; c < 3; c++) { p[c] += vert[3 * v + c]; }
                     }
               for (int c = 0; c < 3; c++) { p[c] /= (double)ids.size(); }
               int id;
               if (ids.size() == 1) { id = ids[0]; }
               else if (ids.size() == 2)
               {
                  auto key = std::make_pair(std::min(ids[0], ids[1]), std::max(ids[0], ids[1]));
                  auto it = edge_mid.find(key);
                  if (it == edge_mid.end()) { id = add_vertex(p); edge_mid.emplace(key, id); }
                  else { id = it->second; }
               }
               else if (ids.size() == 4)
               {
                  std::array<int, 4> key = {ids[0], ids[1], ids[2], ids[3]};
                  std::sort(key.begin(), key.end());
                  auto it = face_mid.find(key);
                  if (it == face_mid.end()) { id = add_vertex(p); face_mid.emplace(key, id); }
                  else { id = it->second; }
               }
               else { id = add_vertex(p); }
               lat[I + 3 * J + 9 * K] = id;
            }
      for (int cz = 0; cz < 2; cz++)
         for (int cy = 0; cy < 2; cy++)
            for (int cx = 0; cx < 2; cx++)
            {
               int child[8];
               for (int a = 0; a < 8; a++)
               {
                  const int ax = a & 1, ay = (a >> 1) & 1, az = a >> 2;
                  child[kLexToNative[a]] = lat[(cx + ax) + 3 * (cy + ay) + 9 * (cz + az)];
               }
               nelem.insert(nelem.end(), child, child + 8);
               nattr.push_back(attr[e]);
            }
   }
   vert.swap(nvert);
   elem.swap(nelem);
   attr.swap(nattr);
   nv = (int)(vert.size() / 3);
   ne = (int)(attr.size());
   if (nx) { nx = 0; ny = 0; nz = 0; }  // element order is no longer lexicographic
}

namespace
{
uint64_t spread3(uint64_t v)  // 21 bits -> every third bit
{
   v &= 0x1fffff;
   v = (v | v << 32) & 0x1f00000000ffffull;
   v = (v | v << 16) & 0x1f0000ff0000ffull;
   v = (v | v << 8) & 0x100f00f00f00f00full;
   v = (v | v << 4) & 0x10c30c30c30c30c3ull;
   v = (v | v << 2) & 0x1249249249249249ull;
   return v;
}

} // namespace

std::vector<int> brick_order(const std::vector<int> &elems, int nx, int ny, int nz)
{
   const int bx = (nx + 3) / 4, by = (ny + 3) / 4, bz = (nz + 3) / 4;
   const long nb = (long)bx * by * bz;
   std::vector<int> count(nb, 0);
   auto key = [&](int e) {
      const int ex = e % nx, ey = (e / nx) % ny, ez = e / (nx * ny);
      return (long)(ex / 4) + bx * ((long)(ey / 4) + (long)by * (ez / 4));
   };
   auto curve = [&](long k) -> uint64_t { return (uint64_t)k; };  // lexicographic brick order
   for (int e : elems) { count[key(e)]++; }
   std::vector<int> out;
   out.reserve(elems.size());
   // complete bricks, in lexicographic brick order, members x-fastest
   std::vector<int> sorted(elems);
   std::stable_sort(sorted.begin(), sorted.end(), [&](int a, int b) {
      const long ka = key(a), kb = key(b);
      if (ka != kb) { return curve(ka) < curve(kb); }
      const int ax = a % nx % 4, ay = (a / nx) % ny % 4, az = (a / (nx * ny)) % 4;
      const int bxx = b % nx % 4, byy = (b / nx) % ny % 4, bzz = (b / (nx * ny)) % 4;
      return ax + 4 * ay + 16 * az < bxx + 4 * byy + 16 * bzz;
   });
   for (int e : sorted) { if (count[key(e)] == 64) { out.push_back(e); } }
   for (int e : elems) { if (count[key(e)] != 64) { out.push_back(e); } }
   return out;
}

std::vector<int> element_order(const HexMesh &m, int kind)
{
   std::vector<int> perm(m.ne);
   for (int e = 0; e < m.ne; e++) { perm[e] = e; }
   if (kind == ORDER_NATIVE || m.ne == 0) { return perm; }
   if (kind == ORDER_BRICK)
   {
      ECM2_VERIFY(m.nx > 0, ERR_ARG, "brick order needs a lexicographic Cartesian mesh");
      return brick_order(perm, m.nx, m.ny, m.nz);
   }
   ECM2_VERIFY(kind == ORDER_MORTON, ERR_ARG, "unknown element order " << kind);
   double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
   std::vector<double> c((size_t)m.ne * 3, 0.0);
   for (int e = 0; e < m.ne; e++)
      for (int k = 0; k < 8; k++)
         for (int d = 0; d < 3; d++) { c[3 * (size_t)e + d] += 0.125 * m.vert[3 * (size_t)m.elem[8 * (size_t)e + k] + d]; }
   for (int e = 0; e < m.ne; e++)
      for (int d = 0; d < 3; d++)
      {
         lo[d] = std::min(lo[d], c[3 * (size_t)e + d]);
         hi[d] = std::max(hi[d], c[3 * (size_t)e + d]);
      }
   auto spread = spread3;
   std::vector<uint64_t> code(m.ne);
   for (int e = 0; e < m.ne; e++)
   {
      uint64_t k = 0;
      for (int d = 0; d < 3; d++)
      {
         const double span = hi[d] > lo[d] ? hi[d] - lo[d] : 1.0;
         const uint64_t q = (uint64_t)((c[3 * (size_t)e + d] - lo[d]) / span * 2097151.0);
         k |= spread(q) << d;
      }
      code[e] = k;
   }
   std::stable_sort(perm.begin(), perm.end(), [&](int a, int b) { return code[a] < code[b]; });
   return perm;
}

void HexMesh::element_nodes(std::vector<double> &out) const
{
   out.resize((size_t)ne * 24);
   for (int e = 0; e < ne; e++)
      for (int c = 0; c < 3; c++)
         for (int a = 0; a < 8; a++)
         {
            out[(size_t)e * 24 + c * 8 + a] = vert[3 * (size_t)elem[8 * e + kLexToNative[a]] + c];
         }
}

namespace
{
struct Key3
{
   int a, b, c;
   bool operator==(const Key3 &o) const { return a == o.a && b == o.b && c == o.c; }
};
struct Key3Hash
{
   size_t operator()(const Key3 &k) const
   {
      uint64_t h = (uint64_t)(uint32_t)k.a * 0x9E3779B97F4A7C15ull;
      h ^= (uint64_t)(uint32_t)k.b + 0x7F4A7C159E3779B9ull + (h << 6) + (h >> 2);
      h ^= (uint64_t)(uint32_t)k.c + 0x94D049BB133111EBull + (h << 6) + (h >> 2);
      return (size_t)h;
   }
};
} // namespace

H1Space H1Space::build(const HexMesh &m, int order, int numbering)
{
   ECM2_VERIFY(order >= 1 && order + 1 <= MAX_D1D, ERR_ARG, "unsupported order " << order);
   H1Space s;
   s.order = order;
   s.ne = m.ne;
   const int p = order, D = p + 1;
   s.nd = D * D * D;
   s.numbering = numbering;
   s.gather_map.resize((size_t)m.ne * s.nd);
   if (numbering == NUMBERING_STRUCTURED)
   {
      ECM2_VERIFY(m.nx > 0, ERR_ARG, "structured numbering needs a Cartesian (lexicographic) mesh");
      const long NX = (long)p * m.nx + 1, NY = (long)p * m.ny + 1, NZ = (long)p * m.nz + 1;
      ECM2_VERIFY(NX * NY * NZ < (1L << 31), ERR_ARG, "too many dofs for int32 indices");
      s.ndofs = (int)(NX * NY * NZ);
      for (int e = 0; e < m.ne; e++)
      {
         const int ex = e % m.nx, ey = (e / m.nx) % m.ny, ez = e / (m.nx * m.ny);
         for (int k = 0; k < D; k++)
            for (int j = 0; j < D; j++)
               for (int i = 0; i < D; i++)
               {
                  const long I = (long)p * ex + i, J = (long)p * ey + j, K = (long)p * ez + k;
                  s.gather_map[(size_t)e * s.nd + (k * D + j) * D + i] = (int)(I + NX * (J + NY * K));
               }
      }
      // boundary dofs: lattice faces
      for (long K = 0; K < NZ; K++)
         for (long J = 0; J < NY; J++)
            for (long I = 0; I < NX; I++)
            {
               if (I == 0 || J == 0 || K == 0 || I == NX - 1 || J == NY - 1 || K == NZ - 1)
               {
                  s.bdr_dofs.push_back((int)(I + NX * (J + NY * K)));
               }
            }
      return s;
   }
   ECM2_VERIFY(numbering == NUMBERING_ENTITY, ERR_ARG, "unknown numbering " << numbering);

   // Entity numbering: edges keyed by (min,max) vertex, faces by their 3 smallest vertices.
   std::unordered_map<uint64_t, int> edge_id;
   std::unordered_map<Key3, int, Key3Hash> face_id;
   std::vector<int> face_count;  // number of elements per face (1 => boundary)
   edge_id.reserve((size_t)m.ne * 4);
   face_id.reserve((size_t)m.ne * 4);
   // Element-local entity tables in lexicographic-corner terms.
   // 12 edges: direction dir, fixed coordinates (a,b) of the other two axes.
   // 6 faces: fixed axis + side.
   std::vector<int> elem_edges((size_t)m.ne * 12), elem_faces((size_t)m.ne * 6);
   auto corner_vid = [&](int e, int cx, int cy, int cz) {
      return m.elem[8 * (size_t)e + kLexToNative[cx + 2 * cy + 4 * cz]];
   };
   for (int e = 0; e < m.ne; e++)
   {
      int le = 0;
      for (int dir = 0; dir < 3; dir++)
         for (int b = 0; b < 2; b++)
            for (int a = 0; a < 2; a++, le++)
            {
               int c0[3], c1[3];
               const int o1 = (dir + 1) % 3, o2 = (dir + 2) % 3;
               c0[dir] = 0; c1[dir] = 1;
               c0[o1] = c1[o1] = a;
               c0[o2] = c1[o2] = b;
               const int v0 = corner_vid(e, c0[0], c0[1], c0[2]);
               const int v1 = corner_vid(e, c1[0], c1[1], c1[2]);
               const uint64_t key = ((uint64_t)(uint32_t)std::min(v0, v1) << 32) |
                                    (uint32_t)std::max(v0, v1);
               auto it = edge_id.find(key);
               int id;
               if (it == edge_id.end()) { id = (int)edge_id.size(); edge_id.emplace(key, id); }
               else { id = it->second; }
               elem_edges[(size_t)e * 12 + le] = id;
            }
      int lf = 0;
      for (int ax = 0; ax < 3; ax++)
         for (int side = 0; side < 2; side++, lf++)
         {
            int ids[4], n = 0;
            const int o1 = (ax + 1) % 3, o2 = (ax + 2) % 3;
            for (int t = 0; t < 2; t++)
               for (int s2 = 0; s2 < 2; s2++)
               {
                  int c[3];
                  c[ax] = side; c[o1] = s2; c[o2] = t;
                  ids[n++] = corner_vid(e, c[0], c[1], c[2]);
               }
            std::sort(ids, ids + 4);
            const Key3 key{ids[0], ids[1], ids[2]};
            auto it = face_id.find(key);
            int id;
            if (it == face_id.end())
            {
               id = (int)face_id.size();
               face_id.emplace(key, id);
               face_count.push_back(0);
            }
            else { id = it->second; }
            face_count[id]++;
            elem_faces[(size_t)e * 6 + lf] = id;
         }
   }
   const long nedges = (long)edge_id.size(), nfaces = (long)face_id.size();
   const long pe = p - 1, pf = (long)(p - 1) * (p - 1), pi = (long)(p - 1) * (p - 1) * (p - 1);
   const long off_e = m.nv, off_f = off_e + nedges * pe, off_i = off_f + nfaces * pf;
   const long total = off_i + (long)m.ne * pi;
   ECM2_VERIFY(total < (1L << 31), ERR_ARG, "too many dofs for int32 indices");
   s.ndofs = (int)total;
   std::vector<char> on_bdr(s.ndofs, 0);

   const int pc = p;  // lattice extent
   for (int e = 0; e < m.ne; e++)
   {
      for (int k = 0; k < D; k++)
         for (int j = 0; j < D; j++)
            for (int i = 0; i < D; i++)
            {
               const int l[3] = {i, j, k};
               int nb = 0;
               for (int c = 0; c < 3; c++) { nb += (l[c] == 0 || l[c] == pc); }
               long gid;
               if (nb == 3)
               {
                  gid = corner_vid(e, i / pc, j / pc, k / pc);
               }
               else if (nb == 2)
               {
                  int dir = 0;
                  for (int c = 0; c < 3; c++) { if (l[c] != 0 && l[c] != pc) { dir = c; } }
                  const int o1 = (dir + 1) % 3, o2 = (dir + 2) % 3;
                  const int a = l[o1] / pc, b = l[o2] / pc;
                  const int le = dir * 4 + b * 2 + a;
                  int c0[3], c1[3];
                  c0[dir] = 0; c1[dir] = 1; c0[o1] = c1[o1] = a; c0[o2] = c1[o2] = b;
                  const int v0 = corner_vid(e, c0[0], c0[1], c0[2]);
                  const int v1 = corner_vid(e, c1[0], c1[1], c1[2]);
                  const int t = (v0 < v1) ? l[dir] : pc - l[dir];   // canonical: from min vertex
                  gid = off_e + (long)elem_edges[(size_t)e * 12 + le] * pe + (t - 1);
               }
               else if (nb == 1)
               {
                  int ax = 0;
                  for (int c = 0; c < 3; c++) { if (l[c] == 0 || l[c] == pc) { ax = c; } }
                  const int side = l[ax] / pc;
                  const int o1 = (ax + 1) % 3, o2 = (ax + 2) % 3;
                  const int lf = ax * 2 + side;
                  // face corners g[s2][t] with s along o1, t along o2
                  int g[2][2];
                  for (int t = 0; t < 2; t++)
                     for (int s2 = 0; s2 < 2; s2++)
                     {
                        int c[3];
                        c[ax] = side; c[o1] = s2; c[o2] = t;
                        g[s2][t] = corner_vid(e, c[0], c[1], c[2]);
                     }
                  // canonical frame: origin = min-id corner, first axis toward the
                  // smaller-id neighbour of the origin
                  int os = 0, ot = 0;
                  for (int t = 0; t < 2; t++)
                     for (int s2 = 0; s2 < 2; s2++)
                     {
                        if (g[s2][t] < g[os][ot]) { os = s2; ot = t; }
                     }
                  const int srel = os ? pc - l[o1] : l[o1];
                  const int trel = ot ? pc - l[o2] : l[o2];
                  const bool s_first = g[1 - os][ot] < g[os][1 - ot];
                  const int ca = s_first ? srel : trel, cb = s_first ? trel : srel;
                  gid = off_f + (long)elem_faces[(size_t)e * 6 + lf] * pf +
                        (ca - 1) + (long)(p - 1) * (cb - 1);
                  if (face_count[elem_faces[(size_t)e * 6 + lf]] == 1) { on_bdr[gid] = 1; }
               }
               else
               {
                  gid = off_i + (long)e * pi + (i - 1) + (long)(p - 1) * ((j - 1) + (long)(p - 1) * (k - 1));
               }
               s.gather_map[(size_t)e * s.nd + (k * D + j) * D + i] = (int)gid;
            }
      // vertex/edge dofs on boundary faces
      for (int lf = 0; lf < 6; lf++)
      {
         if (face_count[elem_faces[(size_t)e * 6 + lf]] != 1) { continue; }
         const int ax = lf / 2, side = lf % 2;
         for (int k = 0; k < D; k++)
            for (int j = 0; j < D; j++)
               for (int i = 0; i < D; i++)
               {
                  const int l[3] = {i, j, k};
                  if (l[ax] != side * pc) { continue; }
                  on_bdr[s.gather_map[(size_t)e * s.nd + (k * D + j) * D + i]] = 1;
               }
      }
   }
   for (int d = 0; d < s.ndofs; d++) { if (on_bdr[d]) { s.bdr_dofs.push_back(d); } }
   return s;
}

void H1Space::dof_coords(const HexMesh &m, std::vector<double> &out) const
{
   const int D = order + 1;
   std::vector<double> nodes(D), w(D);
   gauss_lobatto(D, nodes.data(), w.data());
   out.assign((size_t)ndofs * 3, 0.0);
   std::vector<double> en;
   m.element_nodes(en);
   for (int e = 0; e < ne; e++)
   {
      const double *X = &en[(size_t)e * 24];
      for (int k = 0; k < D; k++)
         for (int j = 0; j < D; j++)
            for (int i = 0; i < D; i++)
            {
               const double xi[3] = {nodes[i], nodes[j], nodes[k]};
               double p[3] = {0, 0, 0};
               for (int a = 0; a < 8; a++)
               {
                  const int ax = a & 1, ay = (a >> 1) & 1, az = a >> 2;
                  const double N = (ax ? xi[0] : 1 - xi[0]) * (ay ? xi[1] : 1 - xi[1]) *
                                   (az ? xi[2] : 1 - xi[2]);
                  for (int c = 0; c < 3; c++) { p[c] += N * X[c * 8 + a]; }
               }
               int g = gather_map[(size_t)e * nd + (k * D + j) * D + i];
               g = g >= 0 ? g : -1 - g;
               for (int c = 0; c < 3; c++) { out[3 * (size_t)g + c] = p[c]; }
            }
   }
}

} // namespace ecm2
