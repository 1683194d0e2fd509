"""Distributed path: y_true = P^T A_local P x_true over an element partition
(RAP, the reference's decomposition), or y_true = R_owned A_local P x_true with ghost elements
(OVERLAP: one exchange per Mult).

CPU (gloo, world_size 2 and 3): every rank builds its local part with the product's
partitioner, applies the ORACLE local operator to its [owned | ghost] L-vector, and runs
the P / P^T exchange with torch.distributed send/recv following the partition's own
neighbour lists -- the same lists the RCCL path uses.  The assembled result must equal
the serial oracle (sum_i P_i^T A_i P_i = A).
GPU (one device): the full partitioned HIP path with the in-process loopback transport."""
import os
import socket

import numpy as np
import pytest

import helpers  # noqa: F401  (registers ecm2_amd in spawned workers too)
import ecm2_amd as E
import oracle as O
from helpers import GOLDEN, RTOL, alpha_bioheat, coeff_function, nonaligned, relerr, temperature


def _mesh(kind):
    if kind in ("cart_big", "bricks"):  # slabs with whole 64-element interior blocks (brick segments)
        m = E.Mesh.MakeCartesian3D(8, 8, 12, 1.0, 1.0, 1.5)
        m.set_vertices(nonaligned(m.vertices()))
        return m
    if kind == "cart":
        m = E.Mesh.MakeCartesian3D(4, 3, 6)
        m.set_vertices(nonaligned(m.vertices()))
        return m
    m = E.Mesh(f"{GOLDEN}/fichera.mesh")
    m.UniformRefinement()
    return m


def _elem_rank(m, kind, nranks):
    if kind in ("cart", "cart_big"):
        return E.partition_slabs_z(m, nranks)
    if kind == "bricks":  # runs of whole 4x4x4 bricks (stepped interfaces, partition_bricks)
        return E.partition_bricks(m, nranks)
    rng = np.random.default_rng(5)  # irregular partition: random element owners
    return rng.integers(0, nranks, m.GetNE()).astype(np.int32)


@pytest.mark.parametrize("kind", ["cart", "fichera", "bricks"])
@pytest.mark.parametrize("nranks", [2, 3, 4])
@pytest.mark.parametrize("decomp", ["rap", "overlap"])
def test_partition_invariants(kind, nranks, decomp):
    m = _mesh(kind)
    fes = E.H1Space(m, 2)
    er = _elem_rank(m, kind, nranks)
    parts = [E.Partition(fes, er, r, nranks, decomposition=decomp) for r in range(nranks)]
    owned = np.concatenate([p.owned_global for p in parts])
    assert np.array_equal(np.sort(owned), np.arange(fes.ndofs))         # each dof owned once
    assert sum(p.ne_owned for p in parts) == fes.ne
    gm = fes.gather_map()
    for p in parts:
        assert p.decomposition == decomp
        if decomp == "rap":
            assert p.ne_local == p.ne_owned
            assert np.all(er[p.elems] == p.rank)
        else:
            # local elements = owned ones + every element touching an owned dof
            own = np.zeros(fes.ndofs, bool)
            own[p.owned_global] = True
            want = np.nonzero((er == p.rank) | own[gm].any(axis=1))[0]
            assert np.array_equal(np.sort(p.elems), want)
            assert int((er[p.elems] == p.rank).sum()) == p.ne_owned
    for p in parts:
        assert np.all(np.diff(p.owned_global) > 0)
        assert np.all(p.gather_map >= 0) and np.all(p.gather_map < p.n_owned + p.n_ghost)
        # interior elements touch no ghost
        assert np.all(p.gather_map[: p.ne_interior] < p.n_owned)
        for k, nb in enumerate(p.nbrs):
            q = parts[nb]
            j = list(q.nbrs).index(p.rank)
            # my ghost block from nb == nb's send block to me (same dofs, same order)
            mine = p.local_to_global[p.n_owned + p.recv_off[k]: p.n_owned + p.recv_off[k + 1]]
            theirs = q.owned_global[q.send_idx[q.send_off[j]: q.send_off[j + 1]]]
            assert np.array_equal(mine, theirs)


def _worker(rank, nranks, port, kind, result_path, decomp="rap"):
    import torch.distributed as dist
    import torch
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=nranks)
    try:
        m = _mesh(kind)
        order = 2
        fes = E.H1Space(m, order)
        er = _elem_rank(m, kind, nranks)
        part = E.Partition(fes, er, rank, nranks, decomposition=decomp)
        q1d = O.default_q1d(order)
        en = m.element_nodes()[part.elems]
        P = O.quad_points(en, q1d)
        c = coeff_function(P)
        nl = part.n_owned + part.n_ghost
        op = O.OracleOperator(en, part.gather_map, nl, order, alpha=c, beta=c)
        xg = np.random.default_rng(0).uniform(-1, 1, fes.ndofs)
        x_true = xg[part.owned_global]
        # P: owner -> ghosts
        xl = np.zeros(nl)
        xl[: part.n_owned] = x_true
        reqs = []
        bufs = []
        for k, nb in enumerate(part.nbrs):
            s = torch.from_numpy(x_true[part.send_idx[part.send_off[k]: part.send_off[k + 1]]].copy())
            r = torch.empty(int(part.recv_off[k + 1] - part.recv_off[k]), dtype=torch.float64)
            bufs.append((k, r))
            if s.numel():
                reqs.append(dist.isend(s, int(nb)))
            if r.numel():
                reqs.append(dist.irecv(r, int(nb)))
        for q in reqs:
            q.wait()
        for k, r in bufs:
            xl[part.n_owned + part.recv_off[k]: part.n_owned + part.recv_off[k + 1]] = r.numpy()
        yl = op.mult(xl)
        y_true = yl[: part.n_owned].copy()
        reqs, bufs = [], []
        # P^T: ghosts -> owners (added); OVERLAP: the owned sums are complete already
        for k, nb in enumerate(part.nbrs if decomp == "rap" else []):
            s = torch.from_numpy(yl[part.n_owned + part.recv_off[k]: part.n_owned + part.recv_off[k + 1]].copy())
            r = torch.empty(int(part.send_off[k + 1] - part.send_off[k]), dtype=torch.float64)
            bufs.append((k, r))
            if s.numel():
                reqs.append(dist.isend(s, int(nb)))
            if r.numel():
                reqs.append(dist.irecv(r, int(nb)))
        for q in reqs:
            q.wait()
        for k, r in bufs:
            np.add.at(y_true, part.send_idx[part.send_off[k]: part.send_off[k + 1]], r.numpy())
        gathered = [None] * nranks
        dist.all_gather_object(gathered, (part.owned_global.tolist(), y_true.tolist()))
        if rank == 0:
            y = np.zeros(fes.ndofs)
            for ids, vals in gathered:
                y[np.array(ids, dtype=np.int64)] = vals
            Pg = O.quad_points(m.element_nodes(), q1d)
            cg = coeff_function(Pg)
            ref = O.OracleOperator(m.element_nodes(), fes.gather_map(), fes.ndofs, order, alpha=cg, beta=cg).mult(xg)
            np.save(result_path, np.array([relerr(y, ref)]))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("kind,nranks", [("cart", 2), ("fichera", 3), ("bricks", 5)])
@pytest.mark.parametrize("decomp", ["rap", "overlap"])
def test_gloo_exchange_matches_serial(tmp_path, kind, nranks, decomp):
    import torch.multiprocessing as mp
    out = str(tmp_path / "err.npy")
    mp.spawn(_worker, args=(nranks, _free_port(), kind, out, decomp), nprocs=nranks, join=True)
    assert float(np.load(out)[0]) <= RTOL


def _schedule_buffers(part, x_true):
    """The five exchange buffers of one rank (par_form.cpp xfer_ptr): x_true, the packed send
    buffer (x_true[send_idx], what kern::gather_idx writes), the ghost blocks of x and y and the
    P^T receive buffer, as numpy arrays a schedule row slices."""
    return {E.Partition.XBUF_X_TRUE: x_true,
            E.Partition.XBUF_SENDBUF: x_true[part.send_idx].copy(),
            E.Partition.XBUF_XGHOST: np.full(part.n_ghost, np.nan),
            E.Partition.XBUF_YGHOST: np.zeros(part.n_ghost),
            E.Partition.XBUF_RECVBUF: np.full(part.send_idx.size, np.nan)}


def _run_schedule(rows, bufs, tag):
    """Issue one exchange exactly as ParPAForm::rccl_exchange does (par_form.cpp:273-286): every
    row of ecm2_partition_exchange_schedule is one send or receive of `count` doubles at
    `offset` of buffer `buf`, to / from `peer`, all posted before any completes (the RCCL group)."""
    import torch
    import torch.distributed as dist
    reqs, landed = [], []
    for peer, send, buf, off, cnt in (tuple(int(v) for v in row) for row in rows):
        if send:
            reqs.append(dist.isend(torch.from_numpy(bufs[buf][off: off + cnt].copy()), peer, tag=tag))
        else:
            t = torch.empty(cnt, dtype=torch.float64)
            reqs.append(dist.irecv(t, peer, tag=tag))
            landed.append((buf, off, t))
    for q in reqs:
        q.wait()
    for buf, off, t in landed:
        bufs[buf][off: off + t.numel()] = t.numpy()


def _worker_schedule(rank, nranks, port, kind, result_path, decomp):
    """One rank of the product's exchange schedule over gloo: the P rows fill the ghost block,
    the oracle applies the local operator, [RAP: the P^T rows carry the ghost contributions into
    the owners' receive buffers, added at send_idx (phase_finish)]."""
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=nranks)
    try:
        m = _mesh(kind)
        order = 2
        fes = E.H1Space(m, order)
        er = _elem_rank(m, kind, nranks)
        part = E.Partition(fes, er, rank, nranks, decomposition=decomp)
        q1d = O.default_q1d(order)
        en = m.element_nodes()[part.elems]
        c = coeff_function(O.quad_points(en, q1d))
        nl = part.n_owned + part.n_ghost
        op = O.OracleOperator(en, part.gather_map, nl, order, alpha=c, beta=c)
        xg = np.random.default_rng(0).uniform(-1, 1, fes.ndofs)
        bufs = _schedule_buffers(part, xg[part.owned_global].copy())
        _run_schedule(part.exchange_schedule(False), bufs, tag=41822)
        assert not np.isnan(bufs[E.Partition.XBUF_XGHOST]).any(), "a ghost was not received"
        yl = op.mult(np.concatenate([bufs[E.Partition.XBUF_X_TRUE], bufs[E.Partition.XBUF_XGHOST]]))
        y_true = yl[: part.n_owned].copy()
        if decomp == "rap":
            bufs[E.Partition.XBUF_YGHOST][:] = yl[part.n_owned:]
            _run_schedule(part.exchange_schedule(True), bufs, tag=41823)
            rb = bufs[E.Partition.XBUF_RECVBUF]
            assert not np.isnan(rb).any(), "a P^T contribution was not received"
            np.add.at(y_true, part.send_idx, rb)
        gathered = [None] * nranks
        dist.all_gather_object(gathered, (part.owned_global.tolist(), y_true.tolist()))
        if rank == 0:
            y = np.zeros(fes.ndofs)
            for ids, vals in gathered:
                y[np.array(ids, dtype=np.int64)] = vals
            cg = coeff_function(O.quad_points(m.element_nodes(), q1d))
            ref = O.OracleOperator(m.element_nodes(), fes.gather_map(), fes.ndofs, order, alpha=cg, beta=cg).mult(xg)
            np.save(result_path, np.array([relerr(y, ref)]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kind,nranks", [("cart", 2), ("cart", 3), ("fichera", 2), ("fichera", 3)])
@pytest.mark.parametrize("decomp", ["rap", "overlap"])
def test_gloo_schedule_rows_match_serial(tmp_path, kind, nranks, decomp):
    """The exact rows the RCCL transport issues (ecm2_partition_exchange_schedule) moved between
    processes: slab (cart: sends straight from x_true) and random (fichera: packed sends)
    partitions, both decompositions; the assembled y equals the serial oracle."""
    import torch.multiprocessing as mp
    out = str(tmp_path / "err.npy")
    mp.spawn(_worker_schedule, args=(nranks, _free_port(), kind, out, decomp), nprocs=nranks, join=True)
    assert float(np.load(out)[0]) <= RTOL


@pytest.mark.gpu
@pytest.mark.parametrize("kind,nranks,order", [("cart", 2, 2), ("cart", 3, 1), ("fichera", 3, 2),
                                               ("fichera", 4, 3), ("cart", 4, 2), ("cart", 2, 4),
                                               ("cart_big", 2, 3), ("cart_big", 3, 4)])
@pytest.mark.parametrize("scatter", ["partials", "atomic"])
@pytest.mark.parametrize("decomp", ["rap", "overlap"])
def test_gpu_loopback_group_matches_serial(kind, nranks, order, scatter, decomp):
    import torch
    m = _mesh(kind)
    fes = E.H1Space(m, order)
    er = _elem_rank(m, kind, nranks)
    q1d = O.default_q1d(order)
    forms, xs, ys, parts = [], [], [], []
    xg = np.random.default_rng(1).uniform(-1, 1, fes.ndofs)
    for r in range(nranks):
        part = E.Partition(fes, er, r, nranks, decomposition=decomp)
        pf = E.ParBilinearForm(part, scatter=scatter)
        P = E.quadrature_points_subset(m, q1d, part.elems)
        c = torch.as_tensor(coeff_function(P).reshape(part.ne_local, -1)).cuda()
        pf.AddDomainIntegrator(E.MassIntegrator(E.QuadratureCoefficient(c)))
        pf.AddDomainIntegrator(E.DiffusionIntegrator(E.QuadratureCoefficient(c.clone())))
        pf.Assemble()
        forms.append(pf)
        parts.append(part)
        xs.append(torch.as_tensor(xg[part.owned_global]).cuda())
        ys.append(torch.full((part.n_owned,), float("nan"), dtype=torch.float64, device="cuda"))
    E.ParGroup(forms).Mult(xs, ys)
    torch.cuda.synchronize()
    y = np.zeros(fes.ndofs)
    for part, yt in zip(parts, ys):
        y[part.owned_global] = yt.cpu().numpy()
    Pg = O.quad_points(m.element_nodes(), q1d)
    cg = coeff_function(Pg)
    ref = O.OracleOperator(m.element_nodes(), fes.gather_map(), fes.ndofs, order, alpha=cg, beta=cg).mult(xg)
    assert relerr(y, ref) <= RTOL


@pytest.mark.gpu
@pytest.mark.parametrize("decomp", ["rap", "overlap"])
@pytest.mark.parametrize("split", ["slabs", "bricks"])
def test_gpu_loopback_group_coefficient_snapshot(decomp, split):
    """slabs: two z-slabs of 4 element layers (RAP: every local block a 4x4x4 lattice-map brick, so
    both take the k(T) snapshot on the split L-vector; OVERLAP adds rank 0 a fifth layer, which keeps
    the stored pairs there).  bricks: partition_bricks of a 12 x 8 x 8 grid into 3 runs of 4 bricks
    (stepped interfaces; whichever layout each rank's blocks allow).  The group Mult matches the
    serial oracle with beta = k(T) projected at the points."""
    import torch
    m = E.Mesh.MakeCartesian3D(8, 8, 8) if split == "slabs" else E.Mesh.MakeCartesian3D(12, 8, 8)
    order = 2
    fes = E.H1Space(m, order)
    nr = 2 if split == "slabs" else 3
    er = E.partition_slabs_z(m, 2) if split == "slabs" else E.partition_bricks(m, 3)
    q1d = O.default_q1d(order)
    T = temperature(fes.dof_coords())
    scale, slope, tref = 0.05, 0.0012, 37.0
    forms, xs, ys, parts = [], [], [], []
    xg = np.random.default_rng(4).uniform(-1, 1, fes.ndofs)
    for r in range(nr):
        part = E.Partition(fes, er, r, nr, decomposition=decomp)
        pf = E.ParBilinearForm(part)
        P = E.quadrature_points_subset(m, q1d, part.elems)
        a = torch.as_tensor(alpha_bioheat(P).reshape(part.ne_local, -1)).cuda()
        Tl = torch.as_tensor(T[part.local_to_global]).cuda()
        pf.AddDomainIntegrator(E.MassIntegrator(E.QuadratureCoefficient(a)))
        pf.AddDomainIntegrator(E.DiffusionIntegrator(E.AffineGridFunctionCoefficient(Tl, scale, slope, tref)))
        pf.Assemble()
        # (OVERLAP: rank 0 holds 5 layers, a leftover layer of non-brick blocks; rank 1's 4 layers are bricks)
        if split == "slabs":
            assert pf.CoefficientSnapshot() == (decomp == "rap" or r == 1)
        else:
            # brick runs (4 whole bricks per rank): with RAP every rank holds bricks only and takes the
            # snapshot (ghost-touching bricks read T' through their lattice map); with OVERLAP the ghost
            # element layers of ranks 0 and 1 are not bricks (profiles/r5/probe_snap_parts.txt)
            assert pf.CoefficientSnapshot() == (decomp == "rap" or r == 2)
        forms.append(pf)
        parts.append(part)
        xs.append(torch.as_tensor(xg[part.owned_global]).cuda())
        ys.append(torch.full((part.n_owned,), float("nan"), dtype=torch.float64, device="cuda"))
    E.ParGroup(forms).Mult(xs, ys)
    torch.cuda.synchronize()
    y = np.zeros(fes.ndofs)
    for part, yt in zip(parts, ys):
        y[part.owned_global] = yt.cpu().numpy()
    en = m.element_nodes()
    Tq = O.interp_evector(T[fes.gather_map()], order, q1d)
    beta = scale * (1.0 + slope * (Tq - tref))
    ref = O.OracleOperator(en, fes.gather_map(), fes.ndofs, order, alpha=alpha_bioheat(O.quad_points(en, q1d)),
                           beta=beta).mult(xg)
    assert relerr(y, ref) <= RTOL


@pytest.mark.gpu
@pytest.mark.parametrize("kind,nranks,order", [("cart", 2, 2), ("fichera", 3, 2), ("fichera", 4, 3),
                                               ("cart_big", 3, 4), ("cart_big", 2, 2)])
@pytest.mark.parametrize("scatter", ["partials", "atomic"])
@pytest.mark.parametrize("decomp", ["rap", "overlap"])
def test_gpu_loopback_overlapped_schedule(kind, nranks, order, scatter, decomp):
    """The overlapped Mult schedule (interior beside exchange + boundary on the comm stream,
    ecm2_par_form_set_schedule) gives the serial oracle's y too."""
    import torch
    m = _mesh(kind)
    fes = E.H1Space(m, order)
    er = _elem_rank(m, kind, nranks)
    q1d = O.default_q1d(order)
    forms, xs, ys, parts = [], [], [], []
    xg = np.random.default_rng(3).uniform(-1, 1, fes.ndofs)
    for r in range(nranks):
        part = E.Partition(fes, er, r, nranks, decomposition=decomp)
        pf = E.ParBilinearForm(part, scatter=scatter, schedule="overlap")
        P = E.quadrature_points_subset(m, q1d, part.elems)
        c = torch.as_tensor(coeff_function(P).reshape(part.ne_local, -1)).cuda()
        pf.AddDomainIntegrator(E.MassIntegrator(E.QuadratureCoefficient(c)))
        pf.AddDomainIntegrator(E.DiffusionIntegrator(E.QuadratureCoefficient(c.clone())))
        pf.Assemble()
        forms.append(pf)
        parts.append(part)
        xs.append(torch.as_tensor(xg[part.owned_global]).cuda())
        ys.append(torch.full((part.n_owned,), float("nan"), dtype=torch.float64, device="cuda"))
    E.ParGroup(forms).Mult(xs, ys)
    torch.cuda.synchronize()
    y = np.zeros(fes.ndofs)
    for part, yt in zip(parts, ys):
        y[part.owned_global] = yt.cpu().numpy()
    Pg = O.quad_points(m.element_nodes(), q1d)
    cg = coeff_function(Pg)
    ref = O.OracleOperator(m.element_nodes(), fes.gather_map(), fes.ndofs, order, alpha=cg, beta=cg).mult(xg)
    assert relerr(y, ref) <= RTOL


@pytest.mark.gpu
@pytest.mark.parametrize("nranks,order", [(2, 2), (3, 2), (8, 2), (3, 4)])
@pytest.mark.parametrize("schedule,decomp", [("serial", "overlap"), ("overlap", "overlap"), ("serial", "rap")])
def test_gpu_group_member_rows(nranks, order, schedule, decomp):
    """ParGroup.MultMember: one member's rows alone (the stages one RCCL rank runs, ghost values
    copied from the peers' x; RAP: + the P^T receive from the peers' ghost sums of a previous
    group Mult) equal the serial oracle's rows; also replayed from a HIP graph (how bench.py
    --member times it); the other members' y stay untouched."""
    import torch
    m = E.Mesh.MakeCartesian3D(6, 5, 16) if nranks == 8 else _mesh("cart_big")
    m.set_vertices(nonaligned(m.vertices()))
    fes = E.H1Space(m, order, E.NUMBERING_STRUCTURED)
    er = E.partition_slabs_z(m, nranks)
    q1d = O.default_q1d(order)
    forms, xs, ys, parts = [], [], [], []
    xg = np.random.default_rng(11).uniform(-1, 1, fes.ndofs)
    for r in range(nranks):
        part = E.Partition(fes, er, r, nranks, decomposition=decomp)
        pf = E.ParBilinearForm(part, schedule=schedule)
        P = E.quadrature_points_subset(m, q1d, part.elems)
        c = torch.as_tensor(coeff_function(P).reshape(part.ne_local, -1)).cuda()
        pf.AddDomainIntegrator(E.MassIntegrator(E.QuadratureCoefficient(c)))
        pf.AddDomainIntegrator(E.DiffusionIntegrator(E.QuadratureCoefficient(c.clone())))
        pf.Assemble()
        forms.append(pf)
        parts.append(part)
        xs.append(torch.as_tensor(xg[part.owned_global]).cuda())
        ys.append(torch.full((part.n_owned,), float("nan"), dtype=torch.float64, device="cuda"))
    Pg = O.quad_points(m.element_nodes(), q1d)
    cg = coeff_function(Pg)
    ref = O.OracleOperator(m.element_nodes(), fes.gather_map(), fes.ndofs, order, alpha=cg, beta=cg).mult(xg)
    group = E.ParGroup(forms)
    if decomp == "rap":
        # a member's RAP rows copy the peers' state of a group Mult on the same x: refused without one
        # (member 0 owns its interface with member 1: its P^T receive copies member 1's y ghost block)
        with pytest.raises(E.ECM2Error):
            group.MultMember(0, xs, ys)
        x2 = [v.clone() for v in xs]
        group.Mult(x2, ys)
        with pytest.raises(E.ECM2Error):
            group.MultMember(0, xs, ys)
        group.Mult(xs, ys)  # the peers' ghost contributions a member's P^T receive copies
        torch.cuda.synchronize()
        for yt in ys:
            yt.fill_(float("nan"))
    for r in range(nranks):
        group.MultMember(r, xs, ys)
        torch.cuda.synchronize()
        assert relerr(ys[r].cpu().numpy(), ref[parts[r].owned_global]) <= RTOL
        for q in range(r + 1, nranks):
            assert torch.isnan(ys[q]).all()
    r = nranks - 1
    ys[r].fill_(float("nan"))
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=torch.cuda.Stream()):
        group.MultMember(r, xs, ys)
    g.replay()
    g.replay()
    torch.cuda.synchronize()
    assert relerr(ys[r].cpu().numpy(), ref[parts[r].owned_global]) <= RTOL


@pytest.mark.gpu
@pytest.mark.parametrize("nranks", [2, 3])
def test_gpu_member_operator_pcg(nranks):
    """Operator(group, member=r) (ecm2_operator_from_par_member, bench.py --pcg-iters with --member):
    member r as one rank's operator -- its Mult is the oracle's rows of r applied to x with every
    peer-owned dof zero (the principal block), and Jacobi-PCG on it (dots through a one-rank RCCL
    all-reduce) solves that block; RAP is refused (its P^T receive needs the peers' group Mult)."""
    import torch
    m = _mesh("cart_big")
    m.set_vertices(nonaligned(m.vertices()))
    order = 2
    fes = E.H1Space(m, order, E.NUMBERING_STRUCTURED)
    er = E.partition_slabs_z(m, nranks)
    q1d = O.default_q1d(order)
    Pg = O.quad_points(m.element_nodes(), q1d)
    cg = coeff_function(Pg)
    oracle = O.OracleOperator(m.element_nodes(), fes.gather_map(), fes.ndofs, order, alpha=cg, beta=cg)

    def group_of(decomp):
        forms, parts = [], []
        for r in range(nranks):
            part = E.Partition(fes, er, r, nranks, decomposition=decomp)
            pf = E.ParBilinearForm(part)
            P = E.quadrature_points_subset(m, q1d, part.elems)
            c = torch.as_tensor(coeff_function(P).reshape(part.ne_local, -1)).cuda()
            pf.AddDomainIntegrator(E.MassIntegrator(E.QuadratureCoefficient(c)))
            pf.AddDomainIntegrator(E.DiffusionIntegrator(E.QuadratureCoefficient(c.clone())))
            pf.Assemble()
            forms.append(pf)
            parts.append(part)
        return E.ParGroup(forms), parts

    group, parts = group_of("overlap")
    rng = np.random.default_rng(5)
    for r in range(nranks):
        op = E.Operator(group, member=r)
        own = parts[r].owned_global
        assert op.size == len(own)
        xl = rng.uniform(-1, 1, len(own))
        xg = np.zeros(fes.ndofs)
        xg[own] = xl
        y = torch.empty(len(own), dtype=torch.float64, device="cuda")
        op.Mult(torch.as_tensor(xl).cuda(), y)
        torch.cuda.synchronize()
        assert relerr(y.cpu().numpy(), oracle.mult(xg)[own]) <= RTOL
        b = torch.as_tensor(rng.uniform(-1, 1, len(own))).cuda()
        x = torch.empty_like(b)
        it, nrm = op.PCG(b, x, rel_tol=1e-11, max_iter=2000, jacobi=True)
        assert 0 < it < 2000
        op.Mult(x, y)
        torch.cuda.synchronize()
        assert relerr(y.cpu().numpy(), b.cpu().numpy()) <= 1e-8
    rap, _ = group_of("rap")
    with pytest.raises(E.ECM2Error):
        E.Operator(rap, member=0)


@pytest.mark.gpu
@pytest.mark.parametrize("order", [2, 4])
def test_gpu_rccl_single_rank_transport(order):
    """The RCCL transport with one rank (ncclCommInitRank, the comm stream and its events,
    ncclAllReduce'd PCG dots, the RCCL diagonal) against the serial form.  Two ranks need
    two GPUs (RCCL refuses two ranks on one device); the exchange itself is covered by the
    loopback group tests and runs at N > 1 in bench.py."""
    import torch
    m = _mesh("cart")
    fes = E.H1Space(m, order)
    er = np.zeros(m.GetNE(), np.int32)
    part = E.Partition(fes, er, 0, 1)
    assert part.n_owned == fes.ndofs and part.n_ghost == 0
    pf = E.ParBilinearForm(part, rccl_id=E.rccl_unique_id())
    q1d = O.default_q1d(order)
    P = E.quadrature_points_subset(m, q1d, part.elems)
    c = torch.as_tensor(coeff_function(P).reshape(part.ne_local, -1)).cuda()
    pf.AddDomainIntegrator(E.MassIntegrator(E.QuadratureCoefficient(c)))
    pf.AddDomainIntegrator(E.DiffusionIntegrator(E.QuadratureCoefficient(c.clone())))
    pf.Assemble()
    Pg = O.quad_points(m.element_nodes(), q1d)
    cg = coeff_function(Pg)
    ref = O.OracleOperator(m.element_nodes(), fes.gather_map(), fes.ndofs, order, alpha=cg, beta=cg)
    xg = np.random.default_rng(2).uniform(-1, 1, fes.ndofs)
    x = torch.as_tensor(xg[part.owned_global]).cuda()
    y = torch.full_like(x, float("nan"))
    for _ in range(3):  # repeated Mults reuse the comm stream and events
        pf.Mult(x, y)
    torch.cuda.synchronize()
    yy = np.zeros(fes.ndofs)
    yy[part.owned_global] = y.cpu().numpy()
    assert relerr(yy, ref.mult(xg)) <= RTOL
    d = torch.empty_like(x)
    pf.AssembleDiagonal(d)
    dd = np.zeros(fes.ndofs)
    dd[part.owned_global] = d.cpu().numpy()
    assert relerr(dd, ref.diagonal()) < 1e-13
    ess = fes.boundary_dofs()
    ess_local = np.nonzero(np.isin(part.owned_global, ess))[0].astype(np.int32)
    b = np.random.default_rng(4).uniform(-1, 1, fes.ndofs)
    sol = torch.empty_like(x)
    it, _ = E.Operator(pf).PCG(torch.as_tensor(b[part.owned_global]).cuda(), sol,
                               ess=torch.as_tensor(ess_local).cuda(), rel_tol=1e-12, max_iter=3000)
    xr, itr, _ = ref.pcg(b, ess, rel_tol=1e-12, max_iter=3000)
    ss = np.zeros(fes.ndofs)
    ss[part.owned_global] = sol.cpu().numpy()
    assert abs(it - itr) <= 2
    assert relerr(ss, xr) < 1e-9


@pytest.mark.gpu
@pytest.mark.parametrize("kind,nranks", [("cart", 2), ("cart", 3), ("fichera", 3)])
@pytest.mark.parametrize("decomp", ["rap", "overlap"])
def test_gpu_rccl_rows_nonempty_schedule(kind, nranks, decomp):
    """The distributed Mult's exchange rows through RCCL itself: every member's
    schedule rows -- sends straight from x (slabs), from the pack buffer (fichera's random
    partition), the P^T rows of RAP -- become grouped ncclSend/ncclRecv of a one-rank
    communicator to itself; on the null stream and replayed from a captured HIP graph."""
    import torch
    m = _mesh(kind)
    order = 2
    fes = E.H1Space(m, order)
    er = _elem_rank(m, kind, nranks)
    q1d = O.default_q1d(order)
    forms, xs, ys, parts = [], [], [], []
    xg = np.random.default_rng(7).uniform(-1, 1, fes.ndofs)
    nrows = 0
    for r in range(nranks):
        part = E.Partition(fes, er, r, nranks, decomposition=decomp)
        nrows += len(part.exchange_schedule(False))
        pf = E.ParBilinearForm(part)
        P = E.quadrature_points_subset(m, q1d, part.elems)
        c = torch.as_tensor(coeff_function(P).reshape(part.ne_local, -1)).cuda()
        pf.AddDomainIntegrator(E.MassIntegrator(E.QuadratureCoefficient(c)))
        pf.AddDomainIntegrator(E.DiffusionIntegrator(E.QuadratureCoefficient(c.clone())))
        pf.Assemble()
        forms.append(pf)
        parts.append(part)
        xs.append(torch.as_tensor(xg[part.owned_global]).cuda())
        ys.append(torch.full((part.n_owned,), float("nan"), dtype=torch.float64, device="cuda"))
    assert nrows > 0
    cg = coeff_function(O.quad_points(m.element_nodes(), q1d))
    ref = O.OracleOperator(m.element_nodes(), fes.gather_map(), fes.ndofs, order, alpha=cg, beta=cg).mult(xg)

    def check():
        y = np.zeros(fes.ndofs)
        for part, yt in zip(parts, ys):
            y[part.owned_global] = yt.cpu().numpy()
        assert relerr(y, ref) <= RTOL

    group = E.ParGroup(forms)
    group.MultRccl(xs, ys)  # null stream (creates the communicator outside any capture)
    torch.cuda.synchronize()
    check()
    for yt in ys:
        yt.fill_(float("nan"))
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=torch.cuda.Stream()):
        group.MultRccl(xs, ys)
    g.replay()
    g.replay()
    torch.cuda.synchronize()
    check()


@pytest.mark.gpu
@pytest.mark.parametrize("graph", [False, True])
def test_gpu_rccl_p2p_graph_capture(graph):
    """RCCL point-to-point (grouped ncclSend/ncclRecv, here a one-rank communicator talking to
    itself) both launched directly and captured in a HIP graph and replayed -- the mechanism
    of the distributed Mult's graph replay."""
    E.load_library()
    assert E.rccl_p2p_selftest(graph, 10201) == 0.0


def _ids(part, row):
    """Global dof ids a schedule row moves, in transfer order."""
    peer, send, buf, off, cnt = (int(v) for v in row)
    if buf == E.Partition.XBUF_X_TRUE:
        return part.owned_global[off: off + cnt]
    if buf in (E.Partition.XBUF_SENDBUF, E.Partition.XBUF_RECVBUF):
        return part.owned_global[part.send_idx[off: off + cnt]]
    assert buf in (E.Partition.XBUF_XGHOST, E.Partition.XBUF_YGHOST)
    return part.local_to_global[part.n_owned + off: part.n_owned + off + cnt]


@pytest.mark.parametrize("kind", ["slabs", "random"])
@pytest.mark.parametrize("nranks", [2, 3, 5, 8])
@pytest.mark.parametrize("decomp", ["rap", "overlap"])
def test_exchange_schedule_pairs(kind, nranks, decomp):
    """The one (peer, buffer, offset, count) schedule both transports consume
    (ecm2_partition_exchange_schedule): the RCCL form issues exactly these ncclSend/ncclRecv
    calls, the loopback group copies each receive from the peer's matching send.  Every send
    of rank r to q has exactly one receive of q from r with the same count, and both move the
    same global dofs in the same order; the P receives tile the ghost block; the P^T sends
    tile it again and the P^T receives cover the P sends (pfespace.cpp:5394-5532)."""
    m = E.Mesh.MakeCartesian3D(6, 5, 16)
    fes = E.H1Space(m, 2, E.NUMBERING_STRUCTURED)
    er = E.partition_slabs_z(m, nranks) if kind == "slabs" else \
        np.random.default_rng(nranks).integers(0, nranks, m.GetNE()).astype(np.int32)
    parts = [E.Partition(fes, er, r, nranks, decomposition=decomp) for r in range(nranks)]
    for transpose in (False, True):
        sch = [p.exchange_schedule(transpose) for p in parts]
        for r, p in enumerate(parts):
            ghosts = np.zeros(p.n_ghost, np.int32)
            for row in sch[r]:
                peer, send, buf, off, cnt = (int(v) for v in row)
                assert peer != r and cnt > 0 and peer in p.nbrs
                if (not transpose and not send) or (transpose and send):
                    assert buf == (E.Partition.XBUF_XGHOST if not transpose else E.Partition.XBUF_YGHOST)
                    ghosts[off: off + cnt] += 1
                if not send:
                    continue
                match = [q for q in sch[peer] if q[0] == r and q[1] == 0]
                assert len(match) == 1 and int(match[0][4]) == cnt
                assert np.array_equal(_ids(p, row), _ids(parts[peer], match[0]))
            assert np.all(ghosts == 1)  # each ghost received (P) / sent back (P^T) exactly once
            if kind == "slabs" and not transpose:
                # z-slabs: every P send is one contiguous owned range, sent straight from x
                assert all(int(row[2]) == E.Partition.XBUF_X_TRUE for row in sch[r] if row[1])


def test_partition_boxes():
    """CartesianPartitioning into px x py x pz boxes (mesh.cpp:8966): every box holds its share,
    each box is one contiguous block of the element lattice, and (1, 1, n) is the z-slab split."""
    m = E.Mesh.MakeCartesian3D(12, 10, 8, 1.0, 10 / 12, 8 / 12)
    r = E.partition_boxes(m, (2, 2, 2))
    assert np.bincount(r).tolist() == [120] * 8
    c = m.element_nodes().mean(axis=2)
    for k in range(8):
        lo, hi = c[r == k].min(axis=0), c[r == k].max(axis=0)
        inside = np.all((c >= lo - 1e-12) & (c <= hi + 1e-12), axis=1)
        assert np.array_equal(inside, r == k)
    assert np.array_equal(E.partition_boxes(m, (1, 1, 4)), E.partition_slabs_z(m, 4))


@pytest.mark.parametrize("dims,nranks", [((12, 8, 8), 3), ((10, 9, 13), 4), ((16, 16, 16), 8), ((5, 4, 4), 2)])
def test_partition_bricks(dims, nranks):
    """partition_bricks: every 4 x 4 x 4 brick of the grid (partial at a ragged edge) lies in one
    part, the parts are runs of the lexicographic brick order and their brick counts differ by
    at most one."""
    m = E.Mesh.MakeCartesian3D(*dims)
    r = E.partition_bricks(m, nranks)
    c = m.element_nodes().mean(axis=2)
    h = 1.0 / np.array(dims, float)
    idx = np.floor(c / h).astype(int)
    nb = [-(-d // 4) for d in dims]
    b = idx // 4
    lin = b[:, 0] + nb[0] * (b[:, 1] + nb[1] * b[:, 2])
    per = {}
    for bl, rr in zip(lin, r):
        per.setdefault(int(bl), set()).add(int(rr))
    assert all(len(v) == 1 for v in per.values())
    owner = np.array([next(iter(per[k])) for k in sorted(per)])
    assert np.all(np.diff(owner) >= 0) and owner[0] == 0 and owner[-1] == nranks - 1
    counts = np.bincount(owner, minlength=nranks)
    assert counts.max() - counts.min() <= 1
    with pytest.raises(E.ECM2Error):
        E.partition_bricks(m, int(np.prod(nb)) + 1)
    # a renumbered (SFC) element order partitions the same elements
    ms = E.Mesh.MakeCartesian3D(*dims, sfc_ordering=True)
    cs = ms.element_nodes().mean(axis=2)
    key = lambda cc: np.lexsort(np.round(cc, 9).T[::-1])
    assert np.array_equal(E.partition_bricks(ms, nranks)[key(cs)], r[key(c)])


def test_partition_boxes_uneven_counts():
    """Counts that do not divide evenly follow the reference's floor(n (c - pmin) / (pmax - pmin))
    (ADVICE r2): 10 elements split 4 ways -> element i in box floor(4 (i + 1/2) / 10); the z-slab
    split of 13 layers into 3 uses the same rule."""
    m = E.Mesh.MakeCartesian3D(10, 3, 13)
    r = E.partition_boxes(m, (4, 1, 1))
    ex = np.arange(m.GetNE()) % 10
    assert np.array_equal(r, np.minimum(3, (2 * ex + 1) * 4 // 20))
    assert r[2] == 1 and r[7] == 3
    ez = np.arange(m.GetNE()) // 30
    want = np.minimum(2, (2 * ez + 1) * 3 // 26)
    assert np.array_equal(E.partition_slabs_z(m, 3), want)
    assert np.array_equal(E.partition_boxes(m, (1, 1, 3)), want)


@pytest.mark.gpu
@pytest.mark.parametrize("decomp", ["rap", "overlap"])
def test_gpu_loopback_group_attribute_markers(decomp):
    """Marked integrators on the distributed form (ParBilinearForm::AddDomainIntegrator(integ,
    marker) on each rank's local elements) give the serial masked operator."""
    import torch
    m = _mesh("fichera")
    m.SetAttributes(1 + np.arange(m.GetNE()) % 2)
    attr = m.GetAttributes()
    order, nranks = 2, 3
    fes = E.H1Space(m, order)
    er = _elem_rank(m, "fichera", nranks)
    q1d = O.default_q1d(order)
    forms, xs, ys, parts = [], [], [], []
    xg = np.random.default_rng(9).uniform(-1, 1, fes.ndofs)
    for r in range(nranks):
        part = E.Partition(fes, er, r, nranks, decomposition=decomp)
        pf = E.ParBilinearForm(part)
        c = torch.as_tensor(coeff_function(E.quadrature_points_subset(m, q1d, part.elems)).reshape(part.ne_local, -1))
        pf.AddDomainIntegrator(E.MassIntegrator(E.QuadratureCoefficient(c.cuda())), [0, 1])
        pf.AddDomainIntegrator(E.DiffusionIntegrator(E.QuadratureCoefficient(c.cuda())))
        pf.Assemble()
        forms.append(pf)
        parts.append(part)
        xs.append(torch.as_tensor(xg[part.owned_global]).cuda())
        ys.append(torch.full((part.n_owned,), float("nan"), dtype=torch.float64, device="cuda"))
    E.ParGroup(forms).Mult(xs, ys)
    torch.cuda.synchronize()
    y = np.zeros(fes.ndofs)
    for part, yt in zip(parts, ys):
        y[part.owned_global] = yt.cpu().numpy()
    cg = coeff_function(O.quad_points(m.element_nodes(), q1d))
    op = O.OracleOperator(m.element_nodes(), fes.gather_map(), fes.ndofs, order, alpha=cg, beta=cg)
    assert relerr(y, op.mult_markers(xg, attr, mass_marker=[0, 1])) <= RTOL


@pytest.mark.gpu
@pytest.mark.parametrize("decomp", ["overlap", "rap"])
def test_gpu_group_member_rows_boxes(decomp):
    """Member emulation on a 2 x 2 x 2 box partition (packed sends, 7 neighbours per rank): each
    member's rows alone equal the serial oracle's, after one group Mult on the same x."""
    import torch
    m = E.Mesh.MakeCartesian3D(8, 8, 8)
    m.set_vertices(nonaligned(m.vertices()))
    fes = E.H1Space(m, 2, E.NUMBERING_STRUCTURED)
    er = E.partition_boxes(m, (2, 2, 2))
    q1d = O.default_q1d(2)
    forms, xs, ys, parts = [], [], [], []
    xg = np.random.default_rng(12).uniform(-1, 1, fes.ndofs)
    for r in range(8):
        part = E.Partition(fes, er, r, 8, decomposition=decomp)
        pf = E.ParBilinearForm(part)
        c = torch.as_tensor(coeff_function(E.quadrature_points_subset(m, q1d, part.elems)).reshape(part.ne_local, -1))
        pf.AddDomainIntegrator(E.MassIntegrator(E.QuadratureCoefficient(c.cuda())))
        pf.AddDomainIntegrator(E.DiffusionIntegrator(E.QuadratureCoefficient(c.cuda())))
        pf.Assemble()
        forms.append(pf)
        parts.append(part)
        xs.append(torch.as_tensor(xg[part.owned_global]).cuda())
        ys.append(torch.full((part.n_owned,), float("nan"), dtype=torch.float64, device="cuda"))
    cg = coeff_function(O.quad_points(m.element_nodes(), q1d))
    ref = O.OracleOperator(m.element_nodes(), fes.gather_map(), fes.ndofs, 2, alpha=cg, beta=cg).mult(xg)
    group = E.ParGroup(forms)
    group.Mult(xs, ys)
    torch.cuda.synchronize()
    for yt in ys:
        yt.fill_(float("nan"))
    for r in range(8):
        group.MultMember(r, xs, ys)
        torch.cuda.synchronize()
        assert relerr(ys[r].cpu().numpy(), ref[parts[r].owned_global]) <= RTOL


def _worker_pcg(rank, nranks, port, kind, result_path, decomp, max_iter):
    """One rank of the product's distributed constrained Jacobi-PCG (pcg_solve, solvers.cpp, with
    ParPAForm as the operator): the Mult is the schedule rows' P exchange + the oracle local
    operator [+ RAP: the P^T rows], the Jacobi diagonal the local diagonal [+ RAP: its P^T sums],
    and every dot is a local partial all-reduced between the processes (ParPAForm::sum_scalars,
    the reference's two MPI_Allreduce per CG iteration: solvers.cpp:931,963, vector.hpp:773-779),
    in pcg_solve's exact step order (the fused x/r/z/r.z update, DIAG_ONE ConstrainedOperator)."""
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=nranks)
    try:
        m = _mesh(kind)
        order = 2
        fes = E.H1Space(m, order)
        er = _elem_rank(m, kind, nranks)
        part = E.Partition(fes, er, rank, nranks, decomposition=decomp)
        q1d = O.default_q1d(order)
        en = m.element_nodes()[part.elems]
        c = coeff_function(O.quad_points(en, q1d))
        nl = part.n_owned + part.n_ghost
        op = O.OracleOperator(en, part.gather_map, nl, order, alpha=c, beta=c)
        tag = [41822]

        def ghost_sums(yl):
            """RAP: the ghost entries' contributions added into their owners (the P^T rows)."""
            y_true = yl[: part.n_owned].copy()
            if decomp == "rap":
                bufs = _schedule_buffers(part, y_true)
                bufs[E.Partition.XBUF_YGHOST][:] = yl[part.n_owned:]
                tag[0] += 1
                _run_schedule(part.exchange_schedule(True), bufs, tag=tag[0])
                np.add.at(y_true, part.send_idx, bufs[E.Partition.XBUF_RECVBUF])
            return y_true

        def mult(x_true):
            bufs = _schedule_buffers(part, x_true.copy())
            tag[0] += 1
            _run_schedule(part.exchange_schedule(False), bufs, tag=tag[0])
            return ghost_sums(op.mult(np.concatenate([x_true, bufs[E.Partition.XBUF_XGHOST]])))

        def allreduce(v):
            t = torch.tensor([v], dtype=torch.float64)
            dist.all_reduce(t)
            return float(t.item())

        own = np.zeros(fes.ndofs, bool)
        own[part.owned_global] = True
        gl = np.full(fes.ndofs, -1, np.int64)
        gl[part.owned_global] = np.arange(part.n_owned)
        ess_g = fes.boundary_dofs()
        ess = gl[ess_g[own[ess_g]]]

        def cmult(v):  # ConstrainedOperator DIAG_ONE: zero ess in place, Mult, restore, out[ess] = in[ess]
            saved = v[ess].copy()
            v[ess] = 0.0
            out = mult(v)
            v[ess] = saved
            out[ess] = saved
            return out

        dg = ghost_sums(op.diagonal())
        dg[ess] = 1.0
        dinv = 1.0 / dg
        b = np.random.default_rng(2).uniform(-1, 1, fes.ndofs)[part.owned_global]
        r = b.copy()
        x = np.zeros(part.n_owned)
        z = dinv * r
        d = z.copy()
        nom = allreduce(d @ r)
        z = cmult(d)
        den = allreduce(z @ d)
        it = 0
        for i in range(1, max_iter + 1):
            alpha = nom / den
            x += alpha * d
            r -= alpha * z
            z = dinv * r
            betanom = allreduce(r @ z)
            it = i
            if i == max_iter:
                break
            d = z + (betanom / nom) * d
            z = cmult(d)
            den = allreduce(d @ z)
            nom = betanom
        gathered = [None] * nranks
        dist.all_gather_object(gathered, (part.owned_global.tolist(), x.tolist(), it))
        if rank == 0:
            xs = np.zeros(fes.ndofs)
            for ids, vals, _ in gathered:
                xs[np.array(ids, dtype=np.int64)] = vals
            cg = coeff_function(O.quad_points(m.element_nodes(), q1d))
            ref = O.OracleOperator(m.element_nodes(), fes.gather_map(), fes.ndofs, order, alpha=cg, beta=cg)
            bg = np.random.default_rng(2).uniform(-1, 1, fes.ndofs)
            xr, itr, _ = ref.pcg(bg, ess_g, rel_tol=0.0, max_iter=max_iter, jacobi=True)
            np.save(result_path, np.array([relerr(xs, xr), it, itr]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kind,nranks", [("cart", 2), ("cart", 3), ("fichera", 2), ("fichera", 3), ("bricks", 3)])
@pytest.mark.parametrize("decomp", ["rap", "overlap"])
def test_gloo_pcg_reductions_match_serial(tmp_path, kind, nranks, decomp):
    """The distributed constrained Jacobi-PCG between processes: the product's step order with
    its two dots per iteration all-reduced over gloo (the RCCL path's ncclAllReduce) and the
    schedule rows' exchange; 8 fixed iterations give the serial oracle CGSolver's iterate."""
    import torch.multiprocessing as mp
    out = str(tmp_path / "pcg.npy")
    mp.spawn(_worker_pcg, args=(nranks, _free_port(), kind, out, decomp, 8), nprocs=nranks, join=True)
    err, it, itr = np.load(out)
    assert it == itr == 8
    assert err < 1e-10
