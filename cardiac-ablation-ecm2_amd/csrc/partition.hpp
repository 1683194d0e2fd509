// partition.hpp -- element partition -> per-rank local space and shared-DoF exchange plan.
//
// Reference: ParMesh / ParFiniteElementSpace (mesh/pmesh.hpp:33, fem/pfespace.cpp) with
// the true-dof prolongation P of DeviceConformingProlongationOperator
// (pfespace.cpp:5259-5532): every shared DoF has one owner rank (here: the lowest rank
// touching it); the true vector of a rank is its owned DoFs; P copies owner values to
// the ghost copies, P^T sums ghost contributions into the owner.
//
// Local L-vector layout: [owned (by global id) | ghost (grouped by owner rank, then by
// global id)], so the true vector is the prefix and each neighbour's ghost block is a
// contiguous range (received in place, sent in place).
//
// Two decompositions:
//  * RAP (the reference's): the rank's local elements are the elements it owns; a Mult is
//    P (owners -> ghost copies), the local PA operator, P^T (ghost contributions summed
//    into the owners).
//  * OVERLAP: the local elements are the owned ones plus every other element touching an
//    owned dof (one element layer per interface); a rank then computes each owned dof's
//    complete sum itself, so a Mult is P, the local operator, and nothing else -- one
//    exchange instead of two, and the owner sums all contributions in a fixed order.  The
//    ghost elements' outputs to non-owned dofs are discarded.  Same y as RAP (any
//    summation order differs only by rounding).
#pragma once

#include "mesh.hpp"

#include <vector>

namespace ecm2
{

struct LocalPart
{
   int rank = 0, nranks = 1, order = 1, nd = 0;
   int ne_local = 0, ne_interior = 0;   // local elements ordered [interior | boundary]
   int ne_owned = 0;                    // elements owned by this rank (ne_local - ghost elements)
   bool overlap = false;                // OVERLAP decomposition (no P^T)
   int n_owned = 0, n_ghost = 0;
   std::vector<int> elems;              // global element ids in local order
   std::vector<int> local_to_global;    // [n_owned + n_ghost]
   std::vector<int> gather_map;         // [ne_local][nd] into the local L-vector
   std::vector<int> nbrs;               // neighbour ranks (ascending)
   std::vector<int> send_off, send_idx; // P: owned local indices sent to nbrs[k] (CSR)
   std::vector<int> recv_off;           // P: ghost block of nbrs[k] = [n_owned+recv_off[k], n_owned+recv_off[k+1])
};

// One point-to-point transfer of an exchange: the unit both transports of the distributed
// form consume (the RCCL form issues one ncclSend / ncclRecv per entry inside one group; the
// in-process loopback group one device copy per receive, from the peer's matching send).
// Buffers of a rank: its true vector x, the packed send buffer, the ghost blocks of x and y,
// the P^T receive buffer; off / count in doubles.
enum XferBuf : int { XBUF_X_TRUE = 0, XBUF_SENDBUF = 1, XBUF_XGHOST = 2, XBUF_YGHOST = 3, XBUF_RECVBUF = 4 };
struct Xfer
{
   int peer, send, buf, off, count;
};
// P (transpose = false, the reference's tag 41822, pfespace.cpp:5394-5440): each neighbour's
// owned interface values -> this rank's ghost block; sent straight from x where the values a
// neighbour needs are one contiguous owned range (z-slabs), else from the packed buffer.  P^T
// (transpose = true, tag 41823, pfespace.cpp:5496-5532): ghost contributions -> the owners'
// receive buffers.  Entries in neighbour order, per neighbour its send before its receive;
// empty transfers are omitted.
std::vector<Xfer> exchange_schedule(const LocalPart &p, bool transpose);

// CartesianPartitioning along z of a Cartesian mesh (any element order; mesh.cpp:8966 semantics
// for a 1 x 1 x nranks grid): elem_rank[e].
std::vector<int> partition_slabs_z(const HexMesh &m, int nranks);

// Equal runs of whole cell^3 bricks of a Cartesian mesh in lexicographic (x-fastest) brick order
// (not a reference partitioner): every part is a union of the bricks the fused kernels assemble,
// balanced to one brick.  elem_rank[e].
std::vector<int> partition_bricks(const HexMesh &m, int nranks, int cell);

// cart (optional): the global mesh when it is Cartesian; interior and boundary element groups
// are then each put in brick order (one 4x4x4 brick per wave).
LocalPart build_local_part(const H1Space &s, const std::vector<int> &elem_rank, int rank, int nranks,
                           const HexMesh *cart = nullptr, bool overlap = false);

} // namespace ecm2
