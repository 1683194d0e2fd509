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

namespace
{
// NCMesh::GridSfcOrdering3D (ncmesh.cpp:5435-5634): the generalized Hilbert ("gilbert") curve
// of a W x H x D box, restated on 3-vectors.  hil(p, a, b, c) walks the box at p spanned by the
// major axis a and the orthogonal axes b, c (each one nonzero component): rows when two extents
// are 1, else halves of the axes (odd halves nudged to even steps) in 2, 3 or 5 sub-boxes.
struct V3
{
   int x, y, z;
   V3 operator+(const V3 &o) const { return {x + o.x, y + o.y, z + o.z}; }
   V3 operator-(const V3 &o) const { return {x - o.x, y - o.y, z - o.z}; }
   V3 operator-() const { return {-x, -y, -z}; }
   V3 half() const { return {x / 2, y / 2, z / 2}; }  // truncation toward zero, as the reference
   int len() const { return std::abs(x + y + z); }
   V3 unit() const { return {(x > 0) - (x < 0), (y > 0) - (y < 0), (z > 0) - (z < 0)}; }
};

void hil(V3 p, V3 a, V3 b, V3 c, std::vector<std::array<int, 3>> &out)
{
   const int w = a.len(), h = b.len(), d = c.len();
   const V3 da = a.unit(), db = b.unit(), dc = c.unit();
   auto row = [&](int n, V3 step) {
      for (int i = 0; i < n; i++, p = p + step) { out.push_back({p.x, p.y, p.z}); }
   };
   if (h == 1 && d == 1) { row(w, da); return; }
   if (w == 1 && d == 1) { row(h, db); return; }
   if (w == 1 && h == 1) { row(d, dc); return; }
   V3 a2 = a.half(), b2 = b.half(), c2 = c.half();
   if ((a2.len() & 1) && w > 2) { a2 = a2 + da; }
   if ((b2.len() & 1) && h > 2) { b2 = b2 + db; }
   if ((c2.len() & 1) && d > 2) { c2 = c2 + dc; }
   if (2 * w > 3 * h && 2 * w > 3 * d)
   {
      hil(p, a2, b, c, out);
      hil(p + a2, a - a2, b, c, out);
   }
   else if (3 * h > 4 * d)
   {
      hil(p, b2, c, a2, out);
      hil(p + b2, a, b - b2, c, out);
      hil(p + (a - da) + (b2 - db), -b2, c, -(a - a2), out);
   }
   else if (3 * d > 4 * h)
   {
      hil(p, c2, a2, b, out);
      hil(p + c2, a, b, c - c2, out);
      hil(p + (a - da) + (c2 - dc), -c2, -(a - a2), b, out);
   }
   else
   {
      hil(p, b2, c2, a2, out);
      hil(p + b2, c, a2, b - b2, out);
      hil(p + (b2 - db) + (c - dc), a, -b2, -(c - c2), out);
      hil(p + (a - da) + b2 + (c - dc), -c, -(a - a2), b - b2, out);
      hil(p + (a - da) + (b2 - db), -b2, c2, -(a - a2), out);
   }
}

std::vector<std::array<int, 3>> grid_sfc_3d(int W, int H, int D)
{
   std::vector<std::array<int, 3>> out;
   out.reserve((size_t)W * H * D);
   const V3 o{0, 0, 0}, X{W, 0, 0}, Y{0, H, 0}, Z{0, 0, D};
   if (W >= H && W >= D) { hil(o, X, Y, Z, out); }
   else if (H >= W && H >= D) { hil(o, Y, X, Z, out); }
   else { hil(o, Z, X, Y, out); }
   return out;
}
} // namespace

HexMesh HexMesh::cartesian(int nx, int ny, int nz, double sx, double sy, double sz, bool sfc_ordering)
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
   std::vector<std::array<int, 3>> order;
   if (sfc_ordering)
   {
      order = grid_sfc_3d(nx, ny, nz);
      ECM2_VERIFY((long)order.size() == (long)m.ne, ERR_INTERNAL, "space-filling curve misses elements");
      m.lex.resize(m.ne);
   }
   for (int e = 0; e < m.ne; e++)
   {
      int x = e % nx, y = (e / nx) % ny, z = e / (nx * ny);  // lexicographic (Make3D without sfc_ordering)
      if (sfc_ordering)
      {
         x = order[e][0]; y = order[e][1]; z = order[e][2];
         m.lex[e] = x + nx * (y + ny * z);
      }
      int *ind = &m.elem[8 * (size_t)e];
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
      return cartesian(nx, ny, nz, sx, sy, sz, true);  // Make3D(..., sfc_ordering = true), mesh_readers.cpp:1506
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

const int kHexEdges[12][2] = {{0, 1}, {1, 2}, {3, 2}, {0, 3}, {4, 5}, {5, 6},
                               {7, 6}, {4, 7}, {0, 4}, {1, 5}, {2, 6}, {3, 7}};
const int kHexFaceVert[6][4] = {{3, 2, 1, 0}, {0, 1, 5, 4}, {1, 2, 6, 5},
                                {2, 3, 7, 6}, {3, 0, 4, 7}, {4, 5, 6, 7}};

HexTopology HexTopology::build(const HexMesh &m)
{
   HexTopology t;
   t.elem_edges.resize((size_t)m.ne * 12);
   t.elem_faces.resize((size_t)m.ne * 6);
   std::unordered_map<uint64_t, int> edge_id;  // (min, max) vertex -> DSTable index
   edge_id.reserve((size_t)m.ne * 4);
   std::unordered_map<Key3, int, Key3Hash> face_id;  // 3 smallest vertices -> STable3D number
   face_id.reserve((size_t)m.ne * 4);
   for (int e = 0; e < m.ne; e++)
   {
      const int *v = &m.elem[8 * (size_t)e];
      for (int k = 0; k < 12; k++)
      {
         const int a = v[kHexEdges[k][0]], b = v[kHexEdges[k][1]];
         const uint64_t key = ((uint64_t)(uint32_t)std::min(a, b) << 32) | (uint32_t)std::max(a, b);
         auto it = edge_id.emplace(key, (int)edge_id.size()).first;
         t.elem_edges[(size_t)e * 12 + k] = it->second;
      }
      for (int k = 0; k < 6; k++)
      {
         int q[4];
         for (int i = 0; i < 4; i++) { q[i] = v[kHexFaceVert[k][i]]; }
         int srt[4] = {q[0], q[1], q[2], q[3]};
         std::sort(srt, srt + 4);
         auto ins = face_id.emplace(Key3{srt[0], srt[1], srt[2]}, (int)face_id.size());
         if (ins.second)
         {
            t.face_vert.insert(t.face_vert.end(), q, q + 4);
            t.face_count.push_back(0);
         }
         t.face_count[ins.first->second]++;
         t.elem_faces[(size_t)e * 6 + k] = ins.first->second;
      }
   }
   t.nedges = (int)edge_id.size();
   t.nfaces = (int)face_id.size();
   return t;
}

void HexMesh::refine_uniform()
{
   // Mesh::UniformRefinement3D_base, hex branch (mesh.cpp:10155-10290, 10635-10705): new
   // vertices at oedge + edge, oface + face, oelem + element (AverageVertices in the tables'
   // vertex order, mesh.cpp:9960; a shared entity is rewritten by every element touching it,
   // the last one's sum stands), each hex -> 8 children with the reference's vertex lists.
   const HexTopology t = HexTopology::build(*this);
   const int oedge = nv, oface = oedge + t.nedges, oelem = oface + t.nfaces;
   std::vector<double> nvert((size_t)(oelem + ne) * 3, 0.0);
   std::copy(vert.begin(), vert.end(), nvert.begin());
   auto average = [&](const int *idx, int n, int result) {
      double acc[3];
      for (int c = 0; c < 3; c++) { acc[c] = vert[3 * (size_t)idx[0] + c]; }
      for (int j = 1; j < n; j++)
         for (int c = 0; c < 3; c++) { acc[c] += vert[3 * (size_t)idx[j] + c]; }
      for (int c = 0; c < 3; c++) { nvert[3 * (size_t)result + c] = acc[c] * (1.0 / n); }
   };
   std::vector<int> nelem((size_t)ne * 64);
   std::vector<int> nattr((size_t)ne * 8);
   for (int i = 0; i < ne; i++)
   {
      const int *v = &elem[8 * (size_t)i];
      const int *E = &t.elem_edges[(size_t)i * 12], *F = &t.elem_faces[(size_t)i * 6];
      average(v, 8, oelem + i);
      for (int fi = 0; fi < 6; fi++)
      {
         int vv[4];
         for (int k = 0; k < 4; k++) { vv[k] = v[kHexFaceVert[fi][k]]; }
         average(vv, 4, oface + F[fi]);
      }
      for (int ei = 0; ei < 12; ei++)
      {
         const int vv[2] = {v[kHexEdges[ei][0]], v[kHexEdges[ei][1]]};
         average(vv, 2, oedge + E[ei]);
      }
      const int c = oelem + i;
      auto e_ = [&](int k) { return oedge + E[k]; };
      auto f_ = [&](int k) { return oface + F[k]; };
      const int kids[8][8] = {
         {v[0], e_(0), f_(0), e_(3), e_(8), f_(1), c, f_(4)},
         {e_(0), v[1], e_(1), f_(0), f_(1), e_(9), f_(2), c},
         {f_(0), e_(1), v[2], e_(2), c, f_(2), e_(10), f_(3)},
         {e_(3), f_(0), e_(2), v[3], f_(4), c, f_(3), e_(11)},
         {e_(8), f_(1), c, f_(4), v[4], e_(4), f_(5), e_(7)},
         {f_(1), e_(9), f_(2), c, e_(4), v[5], e_(5), f_(5)},
         {c, f_(2), e_(10), f_(3), f_(5), e_(5), v[6], e_(6)},
         {f_(4), c, f_(3), e_(11), e_(7), f_(5), e_(6), v[7]}};
      for (int k = 0; k < 8; k++)
      {
         std::copy(kids[k], kids[k] + 8, &nelem[((size_t)i * 8 + k) * 8]);
         nattr[(size_t)i * 8 + k] = attr[i];
      }
   }
   vert.swap(nvert);
   elem.swap(nelem);
   attr.swap(nattr);
   nv = (int)(vert.size() / 3);
   ne = (int)attr.size();
   nx = ny = nz = 0;  // element order is no longer a lattice's
   lex.clear();
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

std::vector<int> brick_order(const std::vector<int> &elems, const HexMesh &m)
{
   const int nx = m.nx, ny = m.ny, nz = m.nz;
   const int bx = (nx + 3) / 4, by = (ny + 3) / 4, bz = (nz + 3) / 4;
   const long nb = (long)bx * by * bz;
   std::vector<int> count(nb, 0);
   auto pos = [&](int e, int &ex, int &ey, int &ez) {
      const int l = m.lex_index(e);
      ex = l % nx; ey = (l / nx) % ny; ez = l / (nx * ny);
   };
   auto key = [&](int e) {
      int ex, ey, ez;
      pos(e, ex, ey, ez);
      return (long)(ex / 4) + bx * ((long)(ey / 4) + (long)by * (ez / 4));
   };
   auto inner = [&](int e) {
      int ex, ey, ez;
      pos(e, ex, ey, ez);
      return ex % 4 + 4 * (ey % 4) + 16 * (ez % 4);
   };
   (void)nb;
   for (int e : elems) { count[key(e)]++; }
   std::vector<int> out;
   out.reserve(elems.size());
   // complete bricks, in lexicographic brick order, members x-fastest
   std::vector<int> sorted(elems);
   std::stable_sort(sorted.begin(), sorted.end(), [&](int a, int b) {
      const long ka = key(a), kb = key(b);
      if (ka != kb) { return ka < kb; }
      return inner(a) < inner(b);
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
      ECM2_VERIFY(m.nx > 0, ERR_ARG, "brick order needs a Cartesian mesh");
      return brick_order(perm, m);
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
      ECM2_VERIFY(m.nx > 0, ERR_ARG, "structured numbering needs a Cartesian mesh");
      const long NX = (long)p * m.nx + 1, NY = (long)p * m.ny + 1, NZ = (long)p * m.nz + 1;
      ECM2_VERIFY(NX * NY * NZ < (1L << 31), ERR_ARG, "too many dofs for int32 indices");
      s.ndofs = (int)(NX * NY * NZ);
      for (int e = 0; e < m.ne; e++)
      {
         const int l = m.lex_index(e), ex = l % m.nx, ey = (l / m.nx) % m.ny, ez = l / (m.nx * m.ny);
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

   // Entity numbering (FiniteElementSpace, fespace.cpp:2767-2860): [vertices | edges (p-1 each) |
   // faces ((p-1)^2 each) | interiors ((p-1)^3 each)], entities in the reference's HexTopology
   // order.  Edge dofs run from the edge's lower vertex id (Mesh::GetElementEdges orientation +
   // DofOrderForOrientation); face dofs are lexicographic in the face's own frame (first
   // element's FaceVert: first axis v0 -> v1, second v0 -> v3); interiors lexicographic.
   const HexTopology t = HexTopology::build(m);
   const long pe = p - 1, pf = (long)(p - 1) * (p - 1), pi = (long)(p - 1) * (p - 1) * (p - 1);
   const long off_e = m.nv, off_f = off_e + (long)t.nedges * pe, off_i = off_f + (long)t.nfaces * pf;
   const long total = off_i + (long)m.ne * pi;
   ECM2_VERIFY(total < (1L << 31), ERR_ARG, "too many dofs for int32 indices");
   s.ndofs = (int)total;
   std::vector<char> on_bdr(s.ndofs, 0);
   const int pc = p;  // lattice extent
   // lexicographic corner (cx, cy, cz) of native vertex n and back
   auto lex_of_native = [](int n, int c) {
      static const int L[8][3] = {{0, 0, 0}, {1, 0, 0}, {1, 1, 0}, {0, 1, 0}, {0, 0, 1}, {1, 0, 1}, {1, 1, 1}, {0, 1, 1}};
      return L[n][c];
   };
   for (int e = 0; e < m.ne; e++)
   {
      const int *v = &m.elem[8 * (size_t)e];
      auto native_of = [&](int gv) {  // native corner of global vertex gv in element e
         for (int n = 0; n < 8; n++) { if (v[n] == gv) { return n; } }
         return -1;
      };
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
                  gid = v[kLexToNative[i / pc + 2 * (j / pc) + 4 * (k / pc)]];
               }
               else if (nb == 2)
               {
                  int dir = 0;
                  for (int c = 0; c < 3; c++) { if (l[c] != 0 && l[c] != pc) { dir = c; } }
                  int c0[3] = {l[0] / pc, l[1] / pc, l[2] / pc}, c1[3] = {c0[0], c0[1], c0[2]};
                  c0[dir] = 0; c1[dir] = 1;
                  const int n0 = kLexToNative[c0[0] + 2 * c0[1] + 4 * c0[2]], n1 = kLexToNative[c1[0] + 2 * c1[1] + 4 * c1[2]];
                  int le = -1;
                  for (int q = 0; q < 12 && le < 0; q++)
                  {
                     if ((kHexEdges[q][0] == n0 && kHexEdges[q][1] == n1) || (kHexEdges[q][0] == n1 && kHexEdges[q][1] == n0)) { le = q; }
                  }
                  const int tt = (v[n0] < v[n1]) ? l[dir] : pc - l[dir];  // from the lower vertex id
                  gid = off_e + (long)t.elem_edges[(size_t)e * 12 + le] * pe + (tt - 1);
               }
               else if (nb == 1)
               {
                  int ax = 0;
                  for (int c = 0; c < 3; c++) { if (l[c] == 0 || l[c] == pc) { ax = c; } }
                  const int side = l[ax] / pc;
                  // local face: the FaceVert entry whose corners all have coordinate `side` on ax
                  int lf = -1;
                  for (int q = 0; q < 6 && lf < 0; q++)
                  {
                     bool ok = true;
                     for (int r = 0; r < 4 && ok; r++) { ok = lex_of_native(kHexFaceVert[q][r], ax) == side; }
                     if (ok) { lf = q; }
                  }
                  const int f = t.elem_faces[(size_t)e * 6 + lf];
                  const int *fv = &t.face_vert[(size_t)f * 4];
                  const int a0 = native_of(fv[0]), a1 = native_of(fv[1]), a3 = native_of(fv[3]);
                  ECM2_VERIFY(a0 >= 0 && a1 >= 0 && a3 >= 0, ERR_INTERNAL, "face frame not on element " << e);
                  // face-frame coordinates of the lattice point: distance from v0 along v0->v1, v0->v3
                  auto along = [&](int from, int to) {
                     int c = 0;
                     for (int q = 0; q < 3; q++) { if (lex_of_native(from, q) != lex_of_native(to, q)) { c = q; } }
                     return lex_of_native(from, c) ? pc - l[c] : l[c];
                  };
                  const int fs = along(a0, a1), ft = along(a0, a3);
                  gid = off_f + (long)f * pf + (fs - 1) + (long)(p - 1) * (ft - 1);
                  if (t.face_count[f] == 1) { on_bdr[gid] = 1; }
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
         if (t.face_count[t.elem_faces[(size_t)e * 6 + lf]] != 1) { continue; }
         const int ax0 = [&] {
            for (int c = 0; c < 3; c++)
            {
               bool same = true;
               for (int r = 1; r < 4; r++) { same &= lex_of_native(kHexFaceVert[lf][r], c) == lex_of_native(kHexFaceVert[lf][0], c); }
               if (same) { return c; }
            }
            return 0;
         }();
         const int side = lex_of_native(kHexFaceVert[lf][0], ax0);
         for (int k = 0; k < D; k++)
            for (int j = 0; j < D; j++)
               for (int i = 0; i < D; i++)
               {
                  const int l[3] = {i, j, k};
                  if (l[ax0] != side * pc) { continue; }
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
