"""GPU parity of the exact forms bench.py times, at the size it times them.

Each case builds its form with bench.py's own `bench_form` (the same mesh, numbering, coefficients,
element order and geometry input as the bench line and its sub-objects) and checks the Mult and the
diagonal against the oracle, with beta = gamma*dt*k(T) of the H1 temperature field interpolated at
the quadrature points -- the reference's setup: GridFunctionCoefficient projection
(qfunction.cpp:73-98, coefficient.cpp:2052-2070) and the law at the point.

Which kernel a case runs is fixed by the form's introspection, asserted here:
* structured numbering, AFFINE + snapshot, every block regular -> k_apply_tpe_ts<3,4,false,RM=1,true>
  (the headline kernel, bench.py's main line);
* the reference's numbering (MakeCartesian3D's SFC element order, entity dofs), AFFINE + snapshot,
  every block a lattice-map block -> k_apply_tpe_ts<3,4,false,RM=3,true> (entity_numbering);
* trilinear mesh, structured -> k_apply_tpe_tlb RM 1 (trilinear); the drop-in configuration
  (entity numbering + trilinear + MFEM Jacobians) -> k_apply_tpe_tlb RM 3 (drop_in);
* configs[4] (68^3, p = 4): AFFINE_E bricks -> k_apply_brick_c (the c5 line).
Bar: ||y - y_ref||_inf / ||y_ref||_inf <= RTOL = 1e-12 (FP64)."""
import importlib.util
import os

import numpy as np
import pytest

import ecm2_amd as E
import oracle as O
from helpers import ROOT, RTOL, relerr

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _bench():
    spec = importlib.util.spec_from_file_location("ecm2_bench", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


B = _bench()


@pytest.fixture(scope="module", autouse=True)
def _device():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    E.load_library()
    yield
    torch.cuda.synchronize()


def host(t):
    torch.cuda.synchronize()
    return t.detach().cpu().numpy()


def _check_form(mesh, fes, form, keep, seed):
    """Mult and diagonal of `form` against the oracle with the bench's coefficients."""
    order, q1d = fes.order, fes.order + 2
    alpha, T = keep[0], keep[1]
    gm = fes.gather_map()
    Tq = O.interp_evector(host(T)[gm], order, q1d)
    beta = B.K_SCALE * (1.0 + B.K_SLOPE * (Tq - B.K_TREF))
    del Tq
    x = np.random.default_rng(seed).uniform(-1, 1, fes.ndofs)
    y = torch.full((fes.ndofs,), float("nan"), dtype=torch.float64, device="cuda")
    form.Mult(torch.as_tensor(x).cuda(), y)
    d = torch.full_like(y, float("nan"))
    form.AssembleDiagonal(d)
    yh, dh = host(y), host(d)
    del y, d
    op = O.OracleOperator(mesh.element_nodes(), gm, fes.ndofs, order, alpha=host(alpha), beta=beta)
    assert relerr(yh, op.mult(x)) <= RTOL
    assert relerr(dh, op.diagonal()) <= RTOL


@pytest.mark.parametrize("n,numbering", [(50, "structured"), (50, "entity"), (108, "structured"), (108, "entity")])
def test_timed_snapshot_forms(n, numbering):
    """configs[3] (108^3, the headline) in both numberings: the k(T) coefficient-snapshot kernel
    k_apply_tpe_ts, RM 1 (structured: every 64-element block a regular lattice brick) or RM 3 (the
    reference's numbering: every block a lattice-map brick).  configs[1] (50^3: 50 is not a
    multiple of the 4-element brick edge, so the last layers are map-read leftover blocks and the
    snapshot does not apply): the stored-pair AFFINE kernel k_apply_tpe_sf with per-block addressing
    (RM 2)."""
    mesh, fes = B.cartesian_space(E, n, n, n, 2, numbering, "affine")
    assert fes.ndofs == (2 * n + 1) ** 3
    keep = []
    form = B.bench_form(E, torch, mesh, fes, keep, element_order="faces" if numbering == "entity" else "auto")
    nblk = (fes.ne + 63) // 64
    assert form.info()["kernel"] == E.KERNEL_TPE and form.info()["layout"] == E.QLAYOUT_AFFINE
    lat, units, _ = form.AddressingInfo()
    lslot, _ = form.PlanInfo()
    assert units == nblk
    if n % 4 == 0:
        assert form.CoefficientSnapshot() and B.qdata_layout(E, form) == "affine_ts"
        if numbering == "structured":
            assert lat == nblk                          # RM 1: every block regular
        else:
            assert lat == 0 and lslot == nblk           # RM 3: every block lattice-mapped
    else:
        assert not form.CoefficientSnapshot() and 0 < lat + lslot < nblk
    _check_form(mesh, fes, form, keep, 100 + n)


@pytest.mark.parametrize("numbering,coefficients", [("structured", "bioheat"), ("entity", "bioheat"),
                                                   ("structured", "pennes")])
def test_snapshot_diagonal_flux_is_the_general_product(monkeypatch, numbering, coefficients):
    """Axis-aligned elements (the Cartesian forms): the snapshot kernel's diagonal flux product
    (k_apply_tpe_ts<..., CD = true>, FluxDiagonal()) gives bit for bit the general product's y
    (ECM2_CDIAG=0 at Assemble), whose off-diagonal terms add exact zeros; a sheared (still affine) mesh
    keeps the general product."""
    order = "faces" if numbering == "entity" else "auto"

    def build(mesh, fes, keep):
        if coefficients == "pennes":
            return B.bench_law_form(E, torch, mesh, fes, keep, "pennes")
        return B.bench_form(E, torch, mesh, fes, keep, element_order=order)

    ys, x = [], None
    for env in ("0", "1"):
        monkeypatch.setenv("ECM2_CDIAG", env)
        mesh, fes = B.cartesian_space(E, 16, 16, 16, 2, numbering, "affine")
        keep = []
        form = build(mesh, fes, keep)
        assert form.CoefficientSnapshot() and form.FluxDiagonal() == (env == "1")
        if x is None:
            x = torch.as_tensor(np.random.default_rng(16).uniform(-1, 1, fes.ndofs)).cuda()
        y = torch.full((fes.ndofs,), float("nan"), dtype=torch.float64, device="cuda")
        form.Mult(x, y)
        ys.append(y)
        if env == "1" and coefficients == "bioheat":
            _check_form(mesh, fes, form, keep, 16)
    assert torch.equal(ys[0], ys[1])
    monkeypatch.delenv("ECM2_CDIAG")
    mesh, fes = B.cartesian_space(E, 16, 16, 16, 2, numbering, "affine")
    v = mesh.vertices()
    v[:, 0] += 0.25 * v[:, 1]
    mesh.set_vertices(v)
    keep = []
    form = build(mesh, fes, keep)
    assert form.CoefficientSnapshot() and not form.FluxDiagonal()
    if coefficients == "bioheat":
        _check_form(mesh, fes, form, keep, 17)


def test_brick_diagonal_flux_is_the_general_product(monkeypatch):
    """The same for the p = 4 brick kernel on AFFINE_E (k_apply_brick_c, G = 3 on axis-aligned elements):
    bit for bit the general product, and the oracle's Mult."""
    ys, x = [], None
    for env in ("0", "1"):
        monkeypatch.setenv("ECM2_CDIAG", env)
        mesh, fes = B.cartesian_space(E, 8, 8, 8, 4, "structured", "affine")
        keep = []
        form = B.bench_form(E, torch, mesh, fes, keep)
        assert form.info()["layout"] == E.QLAYOUT_AFFINE_E and form.FluxDiagonal() == (env == "1")
        if x is None:
            x = torch.as_tensor(np.random.default_rng(8).uniform(-1, 1, fes.ndofs)).cuda()
        y = torch.full((fes.ndofs,), float("nan"), dtype=torch.float64, device="cuda")
        form.Mult(x, y)
        ys.append(y)
        if env == "1":
            _check_form(mesh, fes, form, keep, 8)
    assert torch.equal(ys[0], ys[1])


@pytest.mark.parametrize("variant", ["trilinear", "drop_in"])
def test_timed_trilinear_forms(variant):
    """configs[3] size, bench.py's trilinear and drop_in sub-objects: interior vertices moved
    (non-affine hexes, TRILINEAR layout, k_apply_tpe_tlb); drop_in adds the reference's numbering
    and the geometry as MFEM's GeometricFactors::JACOBIANS (fitted to trilinear maps)."""
    numbering = "entity" if variant == "drop_in" else "structured"
    mesh, fes = B.cartesian_space(E, 108, 108, 108, 2, numbering, "trilinear")
    keep = []
    form = B.bench_form(E, torch, mesh, fes, keep, element_order="faces" if numbering == "entity" else "auto",
                        geometry_input="jacobians" if variant == "drop_in" else "nodes")
    assert form.info()["layout"] == E.QLAYOUT_TRILINEAR and not form.CoefficientSnapshot()
    lat, units, _ = form.AddressingInfo()
    lslot, _ = form.PlanInfo()
    assert (lat == units) if numbering == "structured" else (lslot == units)
    _check_form(mesh, fes, form, keep, 7)


def test_timed_c5_form():
    """configs[4] as bench.py --workload c5 times it: Cartesian 68^3, p = 4 (20.3M DoF), AFFINE_E,
    every element in a lattice-addressed 2 x 2 x 1 brick (k_apply_brick_c<5,6,1,false,1,true>), the
    stored (W beta, W alpha det J) pairs (the bricks do not take the k(T) snapshot: measured slower,
    profiles/r5/ab_c5.txt) and the run-plan summation pass."""
    mesh, fes = B.cartesian_space(E, 68, 68, 68, 4, "structured", "affine")
    assert fes.ndofs == 20346417
    keep = []
    form = B.bench_form(E, torch, mesh, fes, keep)
    assert form.info()["kernel"] == E.KERNEL_LINE and form.info()["layout"] == E.QLAYOUT_AFFINE_E
    assert form.BrickInfo() == (fes.ne // 4, 1) and form.AddressingInfo()[0] == fes.ne // 4
    assert form.SnapshotInfo() == (False, 0, False)
    _check_form(mesh, fes, form, keep, 68)
