"""CPU tests of the product's host side: the C-ABI library loads and exports the
declared symbols, and the setup logic (mesh ingest, refinement, H1 numbering,
boundary dofs) is correct.  No compute entry point runs here (no GPU)."""
import ctypes

import numpy as np
import pytest

import ecm2_amd as E
import oracle as O
from helpers import GOLDEN, element_nodes_from, nonaligned, read_mfem_mesh, relerr


def test_library_exports_every_declared_symbol():
    lib = E.load_library()
    names = E.declared_symbols()
    assert len(names) >= 30
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_compute_entry_points_fail_loudly_without_gpu():
    """No CPU fallback: creating a PA form without a device must raise ECM2_ERR_HIP."""
    lib = E.load_library()
    if lib.ecm2_device_count() > 0:
        pytest.skip("a GPU is visible")
    gm = np.zeros((1, 8), np.int32)
    h = ctypes.c_void_p()
    rc = lib.ecm2_pa_form_create(1, 1, 1, ctypes.c_void_p(gm.ctypes.data), 0, ctypes.byref(h))
    assert rc == 2  # ECM2_ERR_HIP
    assert b"no HIP device" in lib.ecm2_last_error()


def test_cartesian_mesh_matches_make3d_layout():
    m = E.Mesh.MakeCartesian3D(3, 2, 2, 1.5, 1.0, 2.0)
    assert (m.GetNV(), m.GetNE()) == (36, 12)
    V, el = m.vertices(), m.elements()
    # vertex (x,y,z) -> x + (nx+1)(y + (ny+1) z), element vertices per Make3D (mesh.cpp:3784-3791)
    assert np.allclose(V[1], [0.5, 0, 0]) and np.allclose(V[4], [0, 0.5, 0])
    assert list(el[0]) == [0, 1, 5, 4, 12, 13, 17, 16]
    en_prod = m.element_nodes()
    en_orc, _, _, _ = O.cartesian_mesh(3, 2, 2, 1.5, 1.0, 2.0, order=1)
    assert np.array_equal(en_prod, en_orc)


@pytest.mark.parametrize("q1d", [3, 4, 6])
def test_mesh_jacobians_match_geometric_factors(q1d):
    """Mesh.jacobians (the GeometricFactors::JACOBIANS array a drop-in binding passes, MFEM layout
    NQ x 3 x 3 x NE) equals the oracle's restatement of mesh.cpp:15220-15273 on a refined
    fichera mesh with moved interior vertices (trilinear hexes)."""
    m = E.Mesh(f"{GOLDEN}/fichera.mesh")
    m.UniformRefinement()
    V = m.vertices()
    V += 0.05 * np.sin(7.0 * V[:, [1, 2, 0]])
    m.set_vertices(V)
    J = m.jacobians(q1d, device="cpu").numpy()
    _, Jr, _ = O.geom(m.element_nodes(), q1d)
    assert J.shape == Jr.shape
    assert relerr(J, Jr) < 1e-14


def test_mesh_readers_against_reference_fixtures():
    """data/fichera.mesh and data/inline-hex.mesh (reference fixtures) parse to the same
    vertices/elements as an independent parser."""
    m = E.Mesh(f"{GOLDEN}/fichera.mesh")
    V, El = read_mfem_mesh(f"{GOLDEN}/fichera.mesh")
    assert np.array_equal(m.vertices(), V) and np.array_equal(m.elements(), El)
    mi = E.Mesh(f"{GOLDEN}/inline-hex.mesh")
    assert (mi.GetNV(), mi.GetNE()) == (125, 64)


@pytest.mark.parametrize("order", [1, 2, 3, 4])
def test_h1_numbering_conforming(order):
    """Every dof gets the same coordinate from every element that holds it, ndofs obeys
    V + (p-1)E + (p-1)^2 F + (p-1)^3 NE, and boundary dofs lie on the boundary."""
    m = E.Mesh(f"{GOLDEN}/fichera.mesh")
    m.UniformRefinement()
    fes = E.H1Space(m, order)
    gm = fes.gather_map()
    en = m.element_nodes()
    nodes, _ = O.gauss_lobatto(order + 1)
    D = order + 1
    coords = fes.dof_coords()
    for k in range(D):
        for j in range(D):
            for i in range(D):
                xi = (nodes[i], nodes[j], nodes[k])
                s = np.zeros((fes.ne, 3))
                for a in range(8):
                    ax, ay, az = a & 1, (a >> 1) & 1, a >> 2
                    N = (xi[0] if ax else 1 - xi[0]) * (xi[1] if ay else 1 - xi[1]) * (xi[2] if az else 1 - xi[2])
                    s += N * en[:, :, a]
                assert np.abs(coords[gm[:, (k * D + j) * D + i]] - s).max() < 1e-12
    assert np.unique(gm).size == fes.ndofs
    # counts: fichera r1 = 56 hexes
    nv = m.GetNV()
    el = m.elements()
    edges = set()
    faces = {}
    for e in el:
        c = [e[i] for i in E_LEX]
        for a, b in EDGES:
            edges.add((min(c[a], c[b]), max(c[a], c[b])))
        for f in FACES:
            key = tuple(sorted(c[i] for i in f))
            faces[key] = faces.get(key, 0) + 1
    p = order
    assert fes.ndofs == nv + (p - 1) * len(edges) + (p - 1) ** 2 * len(faces) + (p - 1) ** 3 * m.GetNE()
    bd = fes.boundary_dofs()
    nb_faces = sum(1 for v in faces.values() if v == 1)
    assert nb_faces == 7 * 4 * 3 * 2 - 0 or nb_faces > 0
    # boundary dofs of the fichera: x, y or z on the outer box [-1,1]^3 or on the notch planes
    bc = coords[bd]
    on = np.zeros(len(bd), bool)
    for c in range(3):
        on |= np.isclose(np.abs(bc[:, c]), 1.0) | np.isclose(bc[:, c], 0.0)
    assert on.all()


E_LEX = [0, 1, 3, 2, 4, 5, 7, 6]
EDGES = [(0, 1), (2, 3), (4, 5), (6, 7), (0, 2), (1, 3), (4, 6), (5, 7), (0, 4), (1, 5), (2, 6), (3, 7)]
FACES = [(0, 2, 4, 6), (1, 3, 5, 7), (0, 1, 4, 5), (2, 3, 6, 7), (0, 1, 2, 3), (4, 5, 6, 7)]


def test_uniform_refinement_preserves_geometry():
    m = E.Mesh(f"{GOLDEN}/fichera.mesh")
    en0 = m.element_nodes()
    m.UniformRefinement()
    assert m.GetNE() == 56
    en1 = m.element_nodes()
    # volume preserved (trilinear fichera hexes are affine cubes)
    def vol(en):
        return np.abs(np.prod(en.max(axis=2) - en.min(axis=2), axis=1)).sum()
    assert abs(vol(en0) - vol(en1)) < 1e-12


@pytest.mark.parametrize("order", [1, 2, 3])
def test_structured_and_entity_numbering_give_same_operator(order):
    """Both numberings describe the same space: the oracle operator agrees dof-by-coordinate."""
    m = E.Mesh.MakeCartesian3D(3, 2, 2)
    m.set_vertices(nonaligned(m.vertices()))
    en = m.element_nodes()
    outs = []
    for num in (E.NUMBERING_ENTITY, E.NUMBERING_STRUCTURED):
        fes = E.H1Space(m, order, num)
        xyz = fes.dof_coords()
        op = O.OracleOperator(en, fes.gather_map(), fes.ndofs, order, alpha=1.0, beta=2.0)
        x = np.sin(3 * xyz[:, 0]) * np.cos(xyz[:, 1]) + xyz[:, 2]
        y = op.mult(x)
        order_idx = np.lexsort(np.round(xyz, 10).T)
        outs.append(y[order_idx])
    assert relerr(outs[0], outs[1]) < 1e-13


def _face_links(fes, perm):
    """Check every complete 64-element block of perm is a 4x4x4 brick whose lanes
    ax + 4 ay + 16 az are linked face to face (entry-by-entry dof equality)."""
    gm = fes.gather_map()
    D = fes.order + 1
    G = gm.reshape(fes.ne, D, D, D)  # [e][dz][dy][dx]
    nb = 0
    for b in range(fes.ne // 64):
        lanes = perm[64 * b: 64 * b + 64]
        ok = True
        for l in range(64):
            ax, ay, az = l % 4, (l // 4) % 4, l // 16
            e = lanes[l]
            if ax < 3:
                ok &= np.array_equal(G[e, :, :, D - 1], G[lanes[l + 1], :, :, 0])
            if ay < 3:
                ok &= np.array_equal(G[e, :, D - 1, :], G[lanes[l + 4], :, 0, :])
            if az < 3:
                ok &= np.array_equal(G[e, D - 1, :, :], G[lanes[l + 16], 0, :, :])
        nb += int(ok)
    return nb


@pytest.mark.parametrize("order", [1, 2])
def test_face_brick_order(order):
    """ecm2_h1space_element_order (the derived order a PA form uses without a caller order):
    a permutation; on fichera refined twice (7 hexes x 4^3) all 448 elements form 7 linked
    bricks; on a Cartesian mesh it finds the mesh's own 4x4x4 bricks."""
    m = E.Mesh(f"{GOLDEN}/fichera.mesh")
    m.UniformRefinement()
    m.UniformRefinement()
    fes = E.H1Space(m, order)
    perm = fes.element_order_faces()
    assert sorted(perm.tolist()) == list(range(fes.ne))
    assert fes.ne == 448 and _face_links(fes, perm) == 7
    c = E.Mesh.MakeCartesian3D(9, 8, 5)
    fc = E.H1Space(c, order)
    perm = fc.element_order_faces()
    assert sorted(perm.tolist()) == list(range(fc.ne))
    assert _face_links(fc, perm) == 2 * 2 * 1
    ref = c.element_order(E.ORDER_BRICK)
    assert sorted(perm[:256].tolist()) == sorted(ref[:256].tolist())


# native hex corner -> lexicographic (x, y, z) and the reference's Geometry::CUBE tables
_NAT = np.array([[0, 0, 0], [1, 0, 0], [1, 1, 0], [0, 1, 0], [0, 0, 1], [1, 0, 1], [1, 1, 1], [0, 1, 1]])
_EDGES = [(0, 1), (1, 2), (3, 2), (0, 3), (4, 5), (5, 6), (7, 6), (4, 7), (0, 4), (1, 5), (2, 6), (3, 7)]
_FACES = [(3, 2, 1, 0), (0, 1, 5, 4), (1, 2, 6, 5), (2, 3, 7, 6), (3, 0, 4, 7), (4, 5, 6, 7)]


def _cells(m):
    """Lattice cell (x, y, z) of every element of a unit-cube Cartesian mesh, from its corners."""
    nx = round(1.0 / np.ptp(m.element_nodes()[0, 0]))
    return np.rint(m.element_nodes().min(axis=2) * nx).astype(int)


@pytest.mark.parametrize("shape", [(4, 4, 4), (6, 5, 7), (8, 3, 2), (3, 9, 4), (5, 4, 12)])
def test_cartesian_sfc_ordering(shape):
    """MakeCartesian3D(..., sfc_ordering=True) / the INLINE reader (Make3D, mesh.cpp:3749-3774;
    NCMesh::GridSfcOrdering3D, ncmesh.cpp:5435-5634): the elements visit every cell once, start at
    the origin and walk a continuous generalized Hilbert curve -- consecutive cells share a face,
    but for the odd-extent corner steps gilbert allows (at most a few diagonal moves) -- and for
    a 2^k cube it is a true Hilbert curve (every step a face step)."""
    nx, ny, nz = shape
    m = E.Mesh.MakeCartesian3D(nx, ny, nz, 1.0, ny / nx, nz / nx, sfc_ordering=True)
    c = _cells(m)
    assert len({tuple(v) for v in c}) == nx * ny * nz
    assert tuple(c[0]) == (0, 0, 0)
    steps = np.abs(np.diff(c, axis=0)).sum(axis=1)
    assert steps.max() <= 3
    assert (steps > 1).sum() <= 8
    if len(set(shape)) == 1 and (nx & (nx - 1)) == 0:
        assert np.all(steps == 1)
    # same vertices as the lexicographic mesh, elements permuted
    lexm = E.Mesh.MakeCartesian3D(nx, ny, nz, 1.0, ny / nx, nz / nx)
    assert np.array_equal(m.vertices(), lexm.vertices())
    assert sorted(map(tuple, m.elements())) == sorted(map(tuple, lexm.elements()))
    # the lattice view still works: brick order and structured numbering
    assert sorted(m.element_order(E.ORDER_BRICK)) == list(range(m.GetNE()))
    f = E.H1Space(m, 2, E.NUMBERING_STRUCTURED)
    assert f.ndofs == (2 * nx + 1) * (2 * ny + 1) * (2 * nz + 1)


def test_inline_reader_uses_sfc_order():
    m = E.Mesh(f"{GOLDEN}/inline-hex.mesh")
    s = E.Mesh.MakeCartesian3D(4, 4, 4, sfc_ordering=True)
    assert np.array_equal(m.elements(), s.elements())


@pytest.mark.parametrize("mesh", ["cart_sfc", "fichera", "fichera_r1"])
def test_entity_numbering_follows_reference_tables(mesh):
    """FiniteElementSpace's H1 numbering (fespace.cpp:2767-2860) over the reference's topology
    tables: vertex dofs are the vertex ids; edge k of element e gets nv + (its first-insertion
    index in GetVertexToVertexTable over elements x Edges, DSTable::Push); faces the STable3D::Push4
    first-insertion index over elements x FaceVert; interiors off_i + e.  Checked at p = 2 (one
    dof per entity) against an independent numpy restatement of those insertion orders."""
    if mesh == "cart_sfc":
        m = E.Mesh.MakeCartesian3D(5, 4, 3, sfc_ordering=True)
    else:
        m = E.Mesh(f"{GOLDEN}/fichera.mesh")
        if mesh == "fichera_r1":
            m.UniformRefinement()
    Ev = m.elements()
    fes = E.H1Space(m, 2)
    gm = fes.gather_map().reshape(-1, 3, 3, 3)  # [e][z][y][x]
    nv = m.GetNV()
    edges, faces = {}, {}
    for e in range(m.GetNE()):
        for a, b in _EDGES:
            edges.setdefault(tuple(sorted((Ev[e, a], Ev[e, b]))), len(edges))
        for fv in _FACES:
            faces.setdefault(tuple(sorted(Ev[e, list(fv)])[:3]), len(faces))
    off_f, off_i = nv + len(edges), nv + len(edges) + len(faces)
    assert fes.ndofs == off_i + m.GetNE()
    for e in range(m.GetNE()):
        for n in range(8):
            x, y, z = 2 * _NAT[n]
            assert gm[e, z, y, x] == Ev[e, n]
        for a, b in _EDGES:
            x, y, z = _NAT[a] + _NAT[b]
            assert gm[e, z, y, x] == nv + edges[tuple(sorted((Ev[e, a], Ev[e, b])))]
        for fv in _FACES:
            x, y, z = _NAT[list(fv)].sum(axis=0) // 2
            assert gm[e, z, y, x] == off_f + faces[tuple(sorted(Ev[e, list(fv)])[:3])]
        assert gm[e, 1, 1, 1] == off_i + e


def test_uniform_refinement_follows_reference_numbering():
    """UniformRefinement3D_base (mesh.cpp:10271-10290, 10673-10704): new vertices oedge + edge,
    oface + face, oelem + element, with the reference's tables' entity numbers; child k of
    element i is element 8 i + k and its corners are the reference's vertex lists."""
    m = E.Mesh(f"{GOLDEN}/fichera.mesh")
    Ev, V = m.elements(), m.vertices()
    edges, faces = {}, {}
    E12 = np.empty((m.GetNE(), 12), int)
    F6 = np.empty((m.GetNE(), 6), int)
    for e in range(m.GetNE()):
        for k, (a, b) in enumerate(_EDGES):
            E12[e, k] = edges.setdefault(tuple(sorted((Ev[e, a], Ev[e, b]))), len(edges))
        for k, fv in enumerate(_FACES):
            F6[e, k] = faces.setdefault(tuple(sorted(Ev[e, list(fv)])[:3]), len(faces))
    nv, ne = m.GetNV(), m.GetNE()
    oe, of, oc = nv, nv + len(edges), nv + len(edges) + len(faces)
    m.UniformRefinement()
    R, VR = m.elements(), m.vertices()
    assert m.GetNV() == oc + ne and m.GetNE() == 8 * ne
    for i in range(ne):
        v, e_, f_, c = Ev[i], oe + E12[i], of + F6[i], oc + i
        assert list(R[8 * i]) == [v[0], e_[0], f_[0], e_[3], e_[8], f_[1], c, f_[4]]
        assert list(R[8 * i + 6]) == [c, f_[2], e_[10], f_[3], f_[5], e_[5], v[6], e_[6]]
        assert np.allclose(VR[c], V[v].mean(axis=0), atol=1e-15)
        assert np.allclose(VR[e_[0]], V[[v[0], v[1]]].mean(axis=0), atol=1e-15)


def test_point_coefficients_are_checked_before_the_gpu():
    """Per-quadrature-point coefficient tensors are validated in the Python mirror before a device
    pointer reaches the kernels (which read [ne][nq][dim] float64): wrong dtype, shape or device is an
    ECM2Error, not a silent misread."""
    torch = pytest.importorskip("torch")
    ne, nq = 6, 27
    for c in (E.QuadratureCoefficient(torch.zeros(ne, nq, dtype=torch.float32)),
              E.QuadratureCoefficient(torch.zeros(ne, nq, dtype=torch.float64)),          # a host tensor
              E.VectorCoefficient(torch.zeros(ne, nq, 3, dtype=torch.float64)),
              E.MatrixCoefficient(torch.zeros(ne, nq, 9, dtype=torch.float64), symmetric=True)):
        with pytest.raises(E.ECM2Error):
            E._integrator_args(c, [], ne, nq)
    # the shape rule itself (a device-independent part of the check)
    with pytest.raises(E.ECM2Error):
        E._check_points(E.VectorCoefficient(None), np.zeros((ne, nq, 3)), ((3,),), ne, nq)
    # the grid-function kinds map to the ABI's kinds without touching the data
    assert E.COEFF_GRIDFUNC == 10 and E.GridFunctionCoefficient(None).T is None
    # ... and their fields are checked the same way: float32, a host tensor, or a field
    # whose length is not the form's L-vector size never reaches the snapshot kernels
    for T in (torch.zeros(125, dtype=torch.float32), torch.zeros(125, dtype=torch.float64), None):
        for c in (E.GridFunctionCoefficient(T), E.AffineGridFunctionCoefficient(T, 1.0, 0.1, 37.0),
                  E.PerfusionCoefficient(T, 1.0, 0.1, 0.5, 0.02, 37.0, 50.0)):
            with pytest.raises(E.ECM2Error):
                E._integrator_args(c, [], ne, nq, 125)
    with pytest.raises(E.ECM2Error):
        E._check_field(E.GridFunctionCoefficient(None), np.zeros(125), 125)
