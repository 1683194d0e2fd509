"""GPU parity of the k(T) coefficient snapshot for every grid-function coefficient kind.

The reference projects a GridFunctionCoefficient at the quadrature points at Assemble
(CoefficientVector::Project, coefficient.cpp:2052-2070 -> QuadratureFunction::ProjectGridFunction,
qfunction.cpp:73-98) and a law composed with it is applied at the point (TransformedCoefficient::Eval,
coefficient.cpp:262).  The snapshot kernel k_apply_tpe_ts does the same from a copy of the field taken
at Assemble:
* GridFunctionCoefficient (ECM2_COEFF_GRIDFUNC: ex16p's kappa + alpha u formed at the dofs,
  examples/ex16p.cpp:450-466) and the affine k(T) law: the law folded into the snapshot's dofs;
* the Pennes perfusion law (nonlinear, with shut-off), or a MassIntegrator whose coefficient is a law
  of the same field: the field itself is interpolated and the laws applied at the point;
* a MassIntegrator with a constant coefficient or a same-field law stores one value per element (no
  per-point stream at all); a quadrature coefficient or another field keeps W alpha det J per point.
Checked against the oracle on the same projection: the Mult, the diagonal, the reference-layout qdata
and the E-vector AddMultPA, at 8^3 in both numberings (regular blocks RM 1 / lattice-map blocks RM 3)
and at configs[2]'s size (fichera refined 6x, 14.9M DoF).  The laws themselves belong to the bioheat
application, which is not in the reference snapshot (parity of the laws unpinned; the projection and
the operator are the reference's)."""
import numpy as np
import pytest

import ecm2_amd as E
import oracle as O
import bioheat as BH
from helpers import GOLDEN, RTOL, alpha_bioheat, relerr, temperature

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module", autouse=True)
def _device():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    E.load_library()
    yield
    torch.cuda.synchronize()


def dev(a, dtype=torch.float64):
    return torch.as_tensor(np.ascontiguousarray(a)).to(device="cuda", dtype=dtype)


def host(t):
    torch.cuda.synchronize()
    return t.detach().cpu().numpy()


K_AFF = (0.05, 0.0012, 37.0)
PERF_MASS = (3.6e6, 0.05 * 3.6e3, 6.4e-3, 0.02, 37.0)      # + t_stop
PERF_DIFF = (0.5, 0.1, 1.0, 0.02, 37.0)                   # the perfusion law as a conductivity


def mid_gap_stop(Tq, lo=45.0, hi=55.0):
    """A shut-down temperature in the middle of a gap of the quadrature temperatures (no point on the
    law's discontinuity, so rounding cannot flip a side)."""
    ts = np.unique(Tq.ravel())
    gaps = np.diff(ts)
    mid = np.argmax(gaps * ((ts[:-1] > lo) & (ts[1:] < hi)))
    return 0.5 * (ts[mid] + ts[mid + 1])


def diff_coeff(kind, Td, t_stop):
    if kind == "gridfunc":
        return E.GridFunctionCoefficient(Td), (lambda Tq: Tq)
    if kind == "affine":
        return E.AffineGridFunctionCoefficient(Td, *K_AFF), (lambda Tq: BH.affine_law(Tq, *K_AFF))
    par = PERF_DIFF + (t_stop,)
    return E.PerfusionCoefficient(Td, *par), (lambda Tq: BH.perfusion_law(Tq, *par))


@pytest.mark.parametrize("numbering", [E.NUMBERING_STRUCTURED, E.NUMBERING_ENTITY])
@pytest.mark.parametrize("dkind", ["gridfunc", "affine", "perfusion"])
@pytest.mark.parametrize("mass", ["none", "quad", "const", "perf_same", "perf_other", "perf_marked"])
def test_snapshot_laws(numbering, dkind, mass):
    n, order = 8, 2
    if numbering == E.NUMBERING_ENTITY:
        m = E.Mesh.MakeCartesian3D(n, n, n, 1.0, 0.7, 1.3, sfc_ordering=True)
    else:
        m = E.Mesh.MakeCartesian3D(n, n, n, 1.0, 0.7, 1.3)
    m.SetAttributes(1 + np.arange(m.GetNE()) % 2)
    fes = E.H1Space(m, order, numbering)
    en = m.element_nodes()
    q1d = O.default_q1d(order)
    gm = fes.gather_map()
    X = fes.dof_coords()
    T = temperature(X)
    T2 = 40.0 + 5.0 * np.sin(3.0 * X[:, 0])          # another field (perf_other)
    Tq = BH.temperature_at_quadrature(T, gm, order, q1d)
    t_stop = mid_gap_stop(Tq)
    attr = m.GetAttributes()
    eo = "faces" if numbering == E.NUMBERING_ENTITY else "auto"
    a_q = alpha_bioheat(O.quad_points(en, q1d))
    forms, keep = {}, []
    for snap in (True, False):
        Td, T2d = dev(T), dev(T2)
        keep += [Td, T2d]
        f = E.BilinearForm(fes, element_order=eo, coefficient_snapshot=snap)
        dc, dlaw = diff_coeff(dkind, Td, t_stop)
        f.AddDomainIntegrator(E.DiffusionIntegrator(dc))
        marker = None
        if mass == "quad":
            mc = E.QuadratureCoefficient(dev(a_q.reshape(fes.ne, -1)))
        elif mass == "const":
            mc = E.ConstantCoefficient(3.6e6)
        elif mass in ("perf_same", "perf_marked"):
            mc = E.PerfusionCoefficient(Td, *(PERF_MASS + (t_stop,)))
            marker = [1, 0] if mass == "perf_marked" else None
        elif mass == "perf_other":
            mc = E.PerfusionCoefficient(T2d, *(PERF_MASS + (1e300,)))
        if mass != "none":
            f.AddDomainIntegrator(E.MassIntegrator(mc), marker)
        f.Assemble()
        forms[snap] = f
    form = forms[True]
    on, mvals, at_pt = form.SnapshotInfo()
    assert on and not forms[False].CoefficientSnapshot()
    want_m = {"none": 0, "quad": 1, "const": 2, "perf_same": 2, "perf_other": 1, "perf_marked": 2}[mass]
    assert mvals == want_m
    assert at_pt == (dkind == "perfusion" or mass in ("perf_same", "perf_marked"))
    # bytes: W beta is never stored; the mass per element (tmass 2) or per point (tmass 1)
    nq, nblk = q1d ** 3, (fes.ne + 63) // 64
    snap_b = 8 * (fes.ndofs if numbering == E.NUMBERING_STRUCTURED else 729 * nblk)
    assert form.qdata_bytes() == 48 * 64 * nblk + {0: 0, 1: 8 * 64 * nblk * nq, 2: 8 * 64 * nblk}[mvals] + snap_b
    # the oracle on the reference's projection
    beta = dlaw(Tq)
    if mass == "none":
        alpha = None
    elif mass == "quad":
        alpha = a_q
    elif mass == "const":
        alpha = 3.6e6
    elif mass == "perf_other":
        alpha = BH.perfusion_law(BH.temperature_at_quadrature(T2, gm, order, q1d), *(PERF_MASS + (1e300,)))
    else:
        alpha = BH.perfusion_law(Tq, *(PERF_MASS + (t_stop,)))
    op = O.OracleOperator(en, gm, fes.ndofs, order, alpha=alpha, beta=beta)
    for t in keep:
        t.fill_(1.0e3)  # after Assemble: the snapshot (and the reference's qdata) keep the old fields
    x = np.random.default_rng(31).uniform(-1, 1, fes.ndofs)
    y = torch.full((fes.ndofs,), float("nan"), dtype=torch.float64, device="cuda")
    form.Mult(dev(x), y)
    marked = mass == "perf_marked"
    want = op.mult_markers(x, attr, mass_marker=[1, 0]) if marked else op.mult(x)
    assert relerr(host(y), want) <= RTOL
    y2 = torch.empty_like(y)
    forms[False].Mult(dev(x), y2)
    assert relerr(host(y), host(y2)) <= 1e-13
    d = torch.full_like(y, float("nan"))
    form.AssembleDiagonal(d)
    dwant = op.diagonal_markers(attr, [("diffusion", None), ("mass", [1, 0])]) if marked else op.diagonal()
    assert relerr(host(d), dwant) < 1e-12
    assert relerr(form.qdata(E.DIFFUSION), op.D) < 1e-12
    if mass not in ("none", "perf_marked"):
        assert relerr(form.qdata(E.MASS)[:, 0, :], op.M) < 1e-13
    xe = np.random.default_rng(32).uniform(-1, 1, (fes.ne, fes.nd))
    ye = torch.zeros(fes.ne * fes.nd, dtype=torch.float64, device="cuda")
    form.IntegratorAddMultPA(E.DIFFUSION, dev(xe), ye)
    assert relerr(host(ye).reshape(fes.ne, fes.nd), O.diffusion_apply(op.B, op.G, op.D, xe)) <= RTOL


@pytest.mark.parametrize("dkind", ["gridfunc", "affine", "perfusion"])
@pytest.mark.parametrize("mass", ["quad", "const", "perf_same", "perf_marked"])
@pytest.mark.parametrize("order", [3, 4, 5])
def test_snapshot_laws_bricks(order, dkind, mass):
    """p = 3..5 (the line-kernel family): every element of a Cartesian mesh in a lattice-addressed
    2 x 2 x 1 brick.  The bricks never take the snapshot (measured slower even with no per-point stream
    left, profiles/r5/ab_c5b.txt): every grid-function kind and law is projected at the points at
    Assemble (k_coeff_line) into the stored pairs.  Mult, diagonal and qdata against the oracle."""
    m = E.Mesh.MakeCartesian3D(6, 4, 4, 1.0, 0.7, 1.3)
    m.SetAttributes(1 + np.arange(m.GetNE()) % 2)
    fes = E.H1Space(m, order, E.NUMBERING_STRUCTURED)
    en = m.element_nodes()
    q1d = O.default_q1d(order)
    gm = fes.gather_map()
    T = temperature(fes.dof_coords())
    Tq = BH.temperature_at_quadrature(T, gm, order, q1d)
    t_stop = mid_gap_stop(Tq)
    attr = m.GetAttributes()
    a_q = alpha_bioheat(O.quad_points(en, q1d))
    forms, keep = {}, []
    for snap in (True, False):
        Td = dev(T)
        keep.append(Td)
        f = E.BilinearForm(fes, coefficient_snapshot=snap)
        dc, dlaw = diff_coeff(dkind, Td, t_stop)
        f.AddDomainIntegrator(E.DiffusionIntegrator(dc))
        marker = [1, 0] if mass == "perf_marked" else None
        mc = {"quad": lambda: E.QuadratureCoefficient(dev(a_q.reshape(fes.ne, -1))),
              "const": lambda: E.ConstantCoefficient(3.6e6)}.get(
            mass, lambda: E.PerfusionCoefficient(Td, *(PERF_MASS + (t_stop,))))()
        f.AddDomainIntegrator(E.MassIntegrator(mc), marker)
        f.Assemble()
        forms[snap] = f
    form = forms[True]
    assert form.info()["layout"] == E.QLAYOUT_AFFINE_E and form.BrickInfo() == (fes.ne // 4, 1)
    assert form.SnapshotInfo() == (False, 0, False) and not forms[False].CoefficientSnapshot()
    alpha = a_q if mass == "quad" else 3.6e6 if mass == "const" else BH.perfusion_law(Tq, *(PERF_MASS + (t_stop,)))
    op = O.OracleOperator(en, gm, fes.ndofs, order, alpha=alpha, beta=dlaw(Tq))
    for t in keep:
        t.fill_(1.0e3)
    x = np.random.default_rng(order).uniform(-1, 1, fes.ndofs)
    y = torch.full((fes.ndofs,), float("nan"), dtype=torch.float64, device="cuda")
    form.Mult(dev(x), y)
    marked = mass == "perf_marked"
    assert relerr(host(y), op.mult_markers(x, attr, mass_marker=[1, 0]) if marked else op.mult(x)) <= RTOL
    y2 = torch.empty_like(y)
    forms[False].Mult(dev(x), y2)
    assert relerr(host(y), host(y2)) <= 1e-13
    d = torch.full_like(y, float("nan"))
    form.AssembleDiagonal(d)
    dwant = op.diagonal_markers(attr, [("diffusion", None), ("mass", [1, 0])]) if marked else op.diagonal()
    assert relerr(host(d), dwant) < 1e-12
    assert relerr(form.qdata(E.DIFFUSION), op.D) < 1e-12
    if not marked:
        assert relerr(form.qdata(E.MASS)[:, 0, :], op.M) < 1e-13


@pytest.mark.parametrize("case", ["pennes", "ex16"])
def test_snapshot_laws_c3_size(case):
    """configs[2]'s mesh (fichera refined 6x, 14.9M DoF, the reference's numbering: lattice-map blocks)
    with the snapshot carrying both coefficients.  pennes: Mass(rho c + gamma dt c_b w_b(T)) and
    Diffusion(gamma dt k(T)) of one temperature field -- the laws at the point, one mass value per
    element, no per-point stream; ex16: ex16p's implicit operator M + dt K(u_alpha_gf) with
    u_alpha_gf = kappa + alpha u formed at the dofs and passed as a GridFunctionCoefficient."""
    m = E.Mesh(f"{GOLDEN}/fichera.mesh")
    for _ in range(6):
        m.UniformRefinement()
    order, q1d = 2, O.default_q1d(2)
    fes = E.H1Space(m, order)
    assert fes.ndofs == 14877441
    gm = fes.gather_map()
    T = temperature(fes.dof_coords())
    form = E.BilinearForm(fes)
    Td = dev(T)
    if case == "pennes":
        Tq = BH.temperature_at_quadrature(T, gm, order, q1d)
        par = PERF_MASS + (mid_gap_stop(Tq),)
        ks = (0.5 * 0.05, 0.0012, 37.0)
        form.AddDomainIntegrator(E.MassIntegrator(E.PerfusionCoefficient(Td, *par)))
        form.AddDomainIntegrator(E.DiffusionIntegrator(E.AffineGridFunctionCoefficient(Td, *ks)))
        alpha, beta = BH.perfusion_law(Tq, *par), BH.affine_law(Tq, *ks)
        del Tq
        want = (True, 2, True)
    else:
        dt, kappa, alpha_u = 0.01, 0.5, 0.01
        ua = kappa + alpha_u * T                       # u_alpha_gf (ex16p.cpp:458-462), at the dofs
        Ud = dev(dt * ua)
        form.AddDomainIntegrator(E.MassIntegrator(E.ConstantCoefficient(1.0)))
        form.AddDomainIntegrator(E.DiffusionIntegrator(E.GridFunctionCoefficient(Ud)))
        alpha, beta = 1.0, BH.temperature_at_quadrature(dt * ua, gm, order, q1d)
        want = (True, 2, False)
    form.Assemble()
    assert form.info()["layout"] == E.QLAYOUT_AFFINE and form.SnapshotInfo() == want
    x = np.random.default_rng(66).uniform(-1, 1, fes.ndofs)
    y = torch.full((fes.ndofs,), float("nan"), dtype=torch.float64, device="cuda")
    form.Mult(dev(x), y)
    d = torch.full_like(y, float("nan"))
    form.AssembleDiagonal(d)
    yh, dh = host(y), host(d)
    del y, d, form
    op = O.OracleOperator(m.element_nodes(), gm, fes.ndofs, order, alpha=alpha, beta=beta)
    assert relerr(yh, op.mult(x)) <= RTOL
    assert relerr(dh, op.diagonal()) <= RTOL
