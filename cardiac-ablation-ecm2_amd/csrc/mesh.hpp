// mesh.hpp -- trilinear hexahedral meshes and the H1 (Gauss-Lobatto) dof numbering.
//
// Setup side of the boundary (reference rows a7/a8 and SURVEY §8(f) rank 4):
//   Mesh::Make3D / MakeCartesian3D     mesh/mesh.cpp:3683-3830 (vertex + element layout)
//   MFEM mesh v1.0 / INLINE readers     mesh/mesh_readers.cpp:1356-1506
//   Mesh::UniformRefinement (hex)       mesh/mesh.cpp:11403
//   FiniteElementSpace dof numbering    fem/fespace.cpp:2767 (vertices, edges, faces, interiors)
//   lexicographic element dof map       fem/restriction.cpp:26-107 (gather_map semantics)
//   Mesh::CartesianPartitioning          mesh/mesh.cpp:8966 (slab split used for multi-GPU)
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace ecm2
{

// Native hex vertex order (MFEM Hexahedron): 0:(0,0,0) 1:(1,0,0) 2:(1,1,0) 3:(0,1,0)
// 4:(0,0,1) 5:(1,0,1) 6:(1,1,1) 7:(0,1,1).  Lexicographic corner a = ax + 2ay + 4az.
extern const int kLexToNative[8];

struct HexMesh
{
   int nv = 0, ne = 0;
   std::vector<double> vert;   // [nv][3]
   std::vector<int> elem;      // [ne][8] native order
   std::vector<int> attr;      // [ne]
   // Cartesian provenance (for the structured numbering); nx = 0 when unstructured.  lex[e] =
   // ex + nx (ey + ny ez), the lattice position of element e (empty: lexicographic order).
   int nx = 0, ny = 0, nz = 0;
   std::vector<int> lex;
   int lex_index(int e) const { return lex.empty() ? e : lex[e]; }

   // Mesh::Make3D (mesh.cpp:3683-3813): vertices lexicographic; elements lexicographic or, with
   // sfc_ordering (MakeCartesian3D's default and the INLINE reader's, mesh_readers.cpp:1506),
   // along NCMesh::GridSfcOrdering3D's generalized Hilbert curve (ncmesh.cpp:5435-5634).
   static HexMesh cartesian(int nx, int ny, int nz, double sx, double sy, double sz, bool sfc_ordering = false);
   static HexMesh read(const std::string &path);
   void refine_uniform();
   // Corner coordinates in lexicographic order: out[e][c][a] (a = lex corner).
   void element_nodes(std::vector<double> &out) const;
};

enum ElementOrder : int
{
   ORDER_NATIVE = 0,   // caller's order
   ORDER_BRICK = 1,    // Cartesian: 4x4x4 bricks (one per 64-lane wave), then the rest
   ORDER_MORTON = 2    // any mesh: Morton (Z-order) of element centroids
};
// Permutation perm[i] = caller element at internal position i.
std::vector<int> element_order(const HexMesh &m, int kind);
// Brick order of a subset of the elements of a lexicographic nx x ny x nz mesh: complete
// 4x4x4 bricks first (members x-fastest), then the remaining elements in given order.
std::vector<int> brick_order(const std::vector<int> &elems, const HexMesh &m);

// The reference's topology tables of a hex mesh (what FiniteElementSpace numbers and
// UniformRefinement refines): edges numbered in first-insertion order of
// Mesh::GetVertexToVertexTable over the elements and their Geometry::CUBE Edges (DSTable::Push,
// mesh.cpp:8304-8366, table.cpp:623), faces in first-insertion order of
// Mesh::GetElementToFaceTable over the elements and their FaceVert (STable3D::Push4,
// mesh.cpp:8774-8840, stable3d.cpp:64-165); a face's own frame is its first element's FaceVert
// order (Mesh::AddQuadFaceElement).
struct HexTopology
{
   int nedges = 0, nfaces = 0;
   std::vector<int> elem_edges;       // [ne][12], Edges order
   std::vector<int> elem_faces;       // [ne][6], FaceVert order
   std::vector<int> face_vert;        // [nfaces][4], the face's frame
   std::vector<int> face_count;       // [nfaces] elements per face (1: boundary)
   static HexTopology build(const HexMesh &m);
};
extern const int kHexEdges[12][2];     // Geometry::Constants<CUBE>::Edges (geom.cpp:1020-1024)
extern const int kHexFaceVert[6][4];   // Geometry::Constants<CUBE>::FaceVert (geom.cpp:1032-1036)

enum Numbering : int
{
   NUMBERING_ENTITY = 0,     // vertex -> edge -> face -> interior in the reference's entity order
                             // (FiniteElementSpace, fespace.cpp:2767-2860; HexTopology)
   NUMBERING_STRUCTURED = 1  // lattice (I + NX(J + NY K)) on a Cartesian mesh
};

struct H1Space
{
   int order = 0, ne = 0, nd = 0, ndofs = 0;
   int numbering = NUMBERING_ENTITY;
   std::vector<int> gather_map;   // [ne][nd] lexicographic, MFEM gather_map semantics
   std::vector<int> bdr_dofs;     // sorted dofs on boundary faces (ess_tdof_list for ess_bdr = all)

   static H1Space build(const HexMesh &m, int order, int numbering);
   // Physical coordinates of every dof (from the element trilinear map at GLL nodes).
   void dof_coords(const HexMesh &m, std::vector<double> &out) const;
};

} // namespace ecm2
