// bricks.hpp -- element groupings the fused kernels assemble on chip, found from the
// element->dof map alone (any conforming hex mesh, any element order).
//
// The reference applies every element independently and sums shared dofs afterwards
// (ElementRestriction::MultTranspose, fem/restriction.cpp:152-186); these groupings let
// the MI355X kernels sum the faces shared inside a group in registers / LDS instead, so
// only the group's surface reaches the second (partial-sum) pass.
#pragma once

#include <vector>

namespace ecm2
{

// n[d][e] = the element whose low face in direction d (local index 0 along d) equals
// element e's high face (index D-1) entry by entry, or -1.  Entry-by-entry equality means
// the two elements' other two local axes agree on that face: a consistent link.
struct FaceNeighbors
{
   std::vector<int> n[3];
   int operator()(int d, int e) const { return e < 0 ? -1 : n[d][e]; }
};
FaceNeighbors face_neighbors(int ne, int D, const std::vector<int> &gmap);

// 4 x 4 x 4 bricks of consistently linked elements, one per 64-element block, members
// x-fastest (lane = ax + 4 ay + 16 az, what the thread-per-element kernel's in-wave face
// assembly expects), bricks along a Morton curve of their cells (per patch, patches in
// order of first element), then every element in no
// brick in its original order.  Lattice coordinates come from a breadth-first walk of the
// face links (per connected patch), so bricks align with the patch's own grid (a refined
// fichera hex is a 64^3 patch).  Returns perm (internal position -> element).
std::vector<int> face_brick_order(int ne, int D, const std::vector<int> &gmap);

// 2 x 2 x bz groups for the p >= 3 brick kernel (bz = 1, 2, or 4 / 8 for the column
// bricks the kernel marches layer by layer): greedy in element order, all internal faces
// linked, every member in the same apply segment seg[e], no orientation signs.  belem: [nbrick][4 bz] (member ex + 2 ey + 4 ez); in_brick marks members.
void find_bricks(int ne, int D, const std::vector<int> &gmap, int bz, const std::vector<int> &seg,
                 std::vector<int> &belem, std::vector<char> &in_brick);

} // namespace ecm2
