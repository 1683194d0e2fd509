"""GPU parity: the HIP path (through the C ABI) against the CPU oracle.

Bar: ||y_gpu - y_oracle||_inf / ||y_oracle||_inf <= RTOL = 1e-12 in FP64,
for every kernel variant, order, mesh and coefficient kind, plus the committed golden
vectors, the reference-shaped pieces (restriction, per-integrator AddMultPA, qdata,
diagonal), the PCG caller, edge cases, and full BASELINE sizes."""
import os

import numpy as np
import pytest

import ecm2_amd as E
import helpers as H
import oracle as O
from helpers import (GOLDEN, RTOL, alpha_bioheat, coeff_function, k_of_T, nonaligned, relerr,
                     temperature)

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module", autouse=True)
def _device():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    E.load_library()
    yield
    torch.cuda.synchronize()


AFFINE_ON = True  # the compressed layout is selected whenever it applies (set_geometry_compression)
XWAVE_ON = True   # cross-wave face assembly in every AFFINE thread-per-element workgroup


def dev(a, dtype=torch.float64):
    return torch.as_tensor(np.ascontiguousarray(a)).to(device="cuda", dtype=dtype)


def host(t):
    torch.cuda.synchronize()
    return t.detach().cpu().numpy()


def make_mesh(name):
    if name == "nonaligned":
        m = E.Mesh.MakeCartesian3D(5, 4, 3)            # 60 elements: not a multiple of 64
        m.set_vertices(nonaligned(m.vertices()))
    elif name == "fichera_r1":
        m = E.Mesh(f"{GOLDEN}/fichera.mesh")
        m.UniformRefinement()                          # 56 elements
    elif name == "inline_hex":
        m = E.Mesh(f"{GOLDEN}/inline-hex.mesh")        # 64 elements
    elif name == "cart_bricks":
        m = E.Mesh.MakeCartesian3D(8, 8, 5, 1.0, 0.8, 0.6)   # 4 complete 4x4x4 bricks + leftovers
        m.set_vertices(nonaligned(m.vertices()))
    elif name == "cart_130":
        m = E.Mesh.MakeCartesian3D(13, 5, 2, 2.0, 1.0, 0.5)  # 130 elements: 3 blocks, ragged
    elif name == "trilinear":
        m = E.Mesh.MakeCartesian3D(8, 6, 5)                  # 240 elements, interior vertices moved:
        V = m.vertices()                                      # genuinely trilinear (non-affine) hexes
        inner = np.all((V > 1e-9) & (V < np.array([1.0, 1.0, 1.0]) - 1e-9), axis=1)
        V[inner] += 0.02 * np.random.default_rng(5).uniform(-1, 1, (int(inner.sum()), 3))
        m.set_vertices(V)
    else:
        raise ValueError(name)
    return m


def build_pair(mesh, order, alpha, beta, kernel=E.KERNEL_AUTO, numbering=E.NUMBERING_ENTITY,
               element_order="auto", scatter="partials", compress_geometry=True, geometry="nodes"):
    """Product form + oracle operator on the same mesh; alpha/beta: 'fn', 'bio', float or None;
    geometry="jacobians": the form gets J at the points through SetJacobians (the drop-in path)."""
    fes = E.H1Space(mesh, order, numbering)
    en = mesh.element_nodes()
    q1d = O.default_q1d(order)
    P = O.quad_points(en, q1d)

    def coeff(spec):
        if spec is None:
            return None, None
        if spec == "fn":
            c = coeff_function(P)
        elif spec == "bio_a":
            c = alpha_bioheat(P)
        elif spec == "bio_b":
            c = k_of_T(temperature(P))
        else:
            return float(spec), E.ConstantCoefficient(float(spec))
        return c, E.QuadratureCoefficient(dev(c.reshape(fes.ne, -1)))

    a_np, a_c = coeff(alpha)
    b_np, b_c = coeff(beta)
    form = E.BilinearForm(fes, kernel=kernel, element_order=element_order, scatter=scatter,
                          compress_geometry=compress_geometry, geometry=geometry)
    if geometry == "jacobians":
        form.SetJacobians(mesh.jacobians(q1d))
    if a_c is not None:
        form.AddDomainIntegrator(E.MassIntegrator(a_c))
    if b_c is not None:
        form.AddDomainIntegrator(E.DiffusionIntegrator(b_c))
    form.Assemble()
    op = O.OracleOperator(en, fes.gather_map(), fes.ndofs, order, alpha=a_np, beta=b_np)
    return fes, form, op


KERNELS = {"tpe": E.KERNEL_TPE, "wpe": E.KERNEL_WPE, "unfused": E.KERNEL_UNFUSED, "line": E.KERNEL_LINE}


@pytest.mark.parametrize("mesh_name", ["nonaligned", "fichera_r1", "inline_hex", "cart_130", "cart_bricks"])
@pytest.mark.parametrize("order", [1, 2, 3, 4])
@pytest.mark.parametrize("kernel", ["tpe", "wpe", "unfused", "line"])
def test_mult_matches_oracle(mesh_name, order, kernel):
    if kernel == "tpe" and order > 2:
        pytest.skip("thread-per-element kernel covers p = 1, 2")
    m = make_mesh(mesh_name)
    fes, form, op = build_pair(m, order, "fn", "fn", kernel=KERNELS[kernel])
    x = np.random.default_rng(order).uniform(-1, 1, fes.ndofs)
    y = torch.empty(fes.ndofs, dtype=torch.float64, device="cuda")
    form.Mult(dev(x), y)
    assert relerr(host(y), op.mult(x)) <= RTOL


@pytest.mark.parametrize("order", [1, 2, 3])
@pytest.mark.parametrize("integ", ["mass", "diffusion", "both"])
def test_single_integrators_and_constants(order, integ):
    m = make_mesh("nonaligned")
    alpha = 2.5 if integ in ("mass", "both") else None
    beta = 0.7 if integ in ("diffusion", "both") else None
    fes, form, op = build_pair(m, order, alpha, beta)
    x = np.random.default_rng(7).uniform(-1, 1, fes.ndofs)
    y = torch.empty(fes.ndofs, dtype=torch.float64, device="cuda")
    form.Mult(dev(x), y)
    assert relerr(host(y), op.mult(x)) <= RTOL


@pytest.mark.parametrize("ctype", [3, 4, 5, 6])
@pytest.mark.parametrize("order", [1, 2, 3, 4])
@pytest.mark.parametrize("mesh_name", ["nonaligned", "trilinear"])
def test_anisotropic_diffusion_coefficients(ctype, order, mesh_name):
    """"H1 PA Coefficient" (test_pa_coeff.cpp:129-272), coeffType 3..6 through the C ABI: vector,
    symmetric-matrix (full per-point layout, the fused kernels), asymmetric and constant general
    matrices (the reference's 9-entry qdata, workgroup-per-element kernel), with a MassIntegrator:
    Mult, diagonal, E-vector AddMultPA and the reference-layout qdata against the oracle (itself
    pinned to full assembly, test_oracle_pins.py)."""
    from helpers import anisotropic_coefficients
    m = make_mesh(mesh_name)
    fes = E.H1Space(m, order)
    en = m.element_nodes()
    q1d = O.default_q1d(order)
    P = O.quad_points(en, q1d)
    beta, dim = anisotropic_coefficients(P, ctype)
    alpha = coeff_function(P)
    if beta.ndim == 1:  # constant
        coef = E.MatrixCoefficient(beta.reshape(3, 3))
    elif dim == 3:
        coef = E.VectorCoefficient(dev(beta.reshape(fes.ne, -1, 3)))
    elif dim == 6:
        full = beta[..., [0, 1, 2, 1, 3, 4, 2, 4, 5]]
        coef = E.MatrixCoefficient(dev(full.reshape(fes.ne, -1, 9)), symmetric=True)
    else:
        coef = E.MatrixCoefficient(dev(beta.reshape(fes.ne, -1, 9)))
    form = E.BilinearForm(fes)
    form.AddDomainIntegrator(E.MassIntegrator(E.QuadratureCoefficient(dev(alpha.reshape(fes.ne, -1)))))
    form.AddDomainIntegrator(E.DiffusionIntegrator(coef))
    form.Assemble()
    info = form.info()
    if dim == 9:
        assert info["layout"] == E.QLAYOUT_NATIVE9 and info["kernel"] == E.KERNEL_WPE
    else:
        assert info["layout"] == (E.QLAYOUT_BLOCKED if order <= 2 else E.QLAYOUT_NATIVE)
    op = O.OracleOperator(en, fes.gather_map(), fes.ndofs, order, alpha=alpha, beta=beta, beta_dim=dim)
    x = np.random.default_rng(17).uniform(-1, 1, fes.ndofs)
    y = torch.empty(fes.ndofs, dtype=torch.float64, device="cuda")
    form.Mult(dev(x), y)
    assert relerr(host(y), op.mult(x)) <= RTOL
    d = torch.empty_like(y)
    form.AssembleDiagonal(d)
    assert relerr(host(d), op.diagonal()) < 1e-13
    assert relerr(form.qdata(E.DIFFUSION), op.D) < 1e-13
    xe = np.random.default_rng(18).uniform(-1, 1, (fes.ne, fes.nd))
    ye = torch.zeros(fes.ne * fes.nd, dtype=torch.float64, device="cuda")
    form.IntegratorAddMultPA(E.DIFFUSION, dev(xe), ye)
    assert relerr(host(ye).reshape(fes.ne, fes.nd), O.diffusion_apply_n(op.B, op.G, op.D, xe)) <= RTOL
    if dim == 9:
        with pytest.raises(E.ECM2Error):  # the fused kernels read symmetric qdata only
            f2 = E.BilinearForm(fes, kernel=E.KERNEL_TPE if order <= 2 else E.KERNEL_LINE)
            f2.AddDomainIntegrator(E.DiffusionIntegrator(coef))
            f2.Assemble()


def _lattice_trilinear(n=8):
    """n^3 Cartesian mesh (complete 4x4x4 bricks only) with moved interior vertices."""
    m = E.Mesh.MakeCartesian3D(n, n, n)
    V = m.vertices()
    inner = np.all((V > 1e-9) & (V < 1.0 - 1e-9), axis=1)
    V[inner] += 0.15 / n * np.random.default_rng(9).uniform(-1, 1, (int(inner.sum()), 3))
    m.set_vertices(V)
    return m


@pytest.mark.parametrize("mesh_name", ["cart_bricks", "nonaligned", "trilinear", "lattice_tri"])
@pytest.mark.parametrize("order", [1, 2, 3, 4])
@pytest.mark.parametrize("geometry", ["nodes", "jacobians"])
def test_diffusion_only_compressed_layouts(mesh_name, order, geometry):
    """A form with only a DiffusionIntegrator (ex16's K, ex16p.cpp:464) keeps the compressed
    geometry: AFFINE (C_e + W beta per point) or TRILINEAR (map coefficients + W beta / det J per
    point), 8 B per point, blocked at p <= 2 and element-ordered (AFFINE_E / TRILINEAR_E, the line
    kernel) at p >= 3 -- Mult, diagonal, E-vector AddMultPA and the reference-layout qdata against
    the oracle.  A mass-only form keeps the BLOCKED mass stream (8 B per point)."""
    m = _lattice_trilinear() if mesh_name == "lattice_tri" else make_mesh(mesh_name)
    fes = E.H1Space(m, order)
    en = m.element_nodes()
    q1d = O.default_q1d(order)
    c = coeff_function(O.quad_points(en, q1d))
    form = E.BilinearForm(fes, geometry=geometry)
    if geometry == "jacobians":
        form.SetJacobians(m.jacobians(q1d))
    form.AddDomainIntegrator(E.DiffusionIntegrator(E.QuadratureCoefficient(dev(c.reshape(fes.ne, -1)))))
    form.Assemble()
    affine = mesh_name in ("cart_bricks", "nonaligned")
    if order <= 2:
        assert form.info()["layout"] == (E.QLAYOUT_AFFINE if affine else E.QLAYOUT_TRILINEAR)
    else:
        assert form.info()["layout"] == (E.QLAYOUT_AFFINE_E if affine else E.QLAYOUT_TRILINEAR_E)
        assert form.qdata_bytes() == 8 * fes.ne * ((6 if affine else 21) + q1d ** 3)
    assert form.qdata_bytes() < 20 * fes.ne * q1d ** 3  # 8 B per point + the per-element geometry
    op = O.OracleOperator(en, fes.gather_map(), fes.ndofs, order, alpha=None, beta=c)
    x = np.random.default_rng(13).uniform(-1, 1, fes.ndofs)
    y = torch.empty(fes.ndofs, dtype=torch.float64, device="cuda")
    form.Mult(dev(x), y)
    assert relerr(host(y), op.mult(x)) <= RTOL
    d = torch.empty_like(y)
    form.AssembleDiagonal(d)
    assert relerr(host(d), op.diagonal()) < 1e-13
    assert relerr(form.qdata(E.DIFFUSION), op.D) < 1e-13
    xe = np.random.default_rng(14).uniform(-1, 1, (fes.ne, fes.nd))
    ye = torch.zeros(fes.ne * fes.nd, dtype=torch.float64, device="cuda")
    form.IntegratorAddMultPA(E.DIFFUSION, dev(xe), ye)
    assert relerr(host(ye).reshape(fes.ne, fes.nd), O.diffusion_apply(op.B, op.G, op.D, xe)) <= RTOL
    if geometry == "nodes" and mesh_name == "trilinear" and order <= 2:
        fm = E.BilinearForm(fes)
        fm.AddDomainIntegrator(E.MassIntegrator(E.QuadratureCoefficient(dev(c.reshape(fes.ne, -1)))))
        fm.Assemble()
        assert fm.info()["layout"] == E.QLAYOUT_BLOCKED
        nq = fm.info()["q1d"] ** 3
        assert fm.qdata_bytes() <= 8 * 64 * 2 * ((nq + 1) // 2) * ((fes.ne + 63) // 64)  # pairs of points
        fm.Mult(dev(x), y)
        assert relerr(host(y), O.OracleOperator(en, fes.gather_map(), fes.ndofs, order, alpha=c).mult(x)) <= RTOL


@pytest.mark.parametrize("numbering", [E.NUMBERING_STRUCTURED, E.NUMBERING_ENTITY])
@pytest.mark.parametrize("mass", [True, False])
def test_trilinear_lattice_kernel(numbering, mass):
    """The two-waves-per-SIMD TRILINEAR kernel (every block a lattice brick: regular blocks with
    the structured numbering, lattice-map blocks with the reference's) against the oracle, with
    and without the MassIntegrator, on the distributed form's split L-vector too."""
    m = _lattice_trilinear(8)
    order = 2
    fes = E.H1Space(m, order, numbering)
    en = m.element_nodes()
    q1d = O.default_q1d(order)
    c = coeff_function(O.quad_points(en, q1d))
    form = E.BilinearForm(fes, element_order="faces" if numbering == E.NUMBERING_ENTITY else "auto")
    if mass:
        form.AddDomainIntegrator(E.MassIntegrator(E.QuadratureCoefficient(dev(c.reshape(fes.ne, -1)))))
    form.AddDomainIntegrator(E.DiffusionIntegrator(E.QuadratureCoefficient(dev(c.reshape(fes.ne, -1)))))
    form.Assemble()
    assert form.info()["layout"] == E.QLAYOUT_TRILINEAR
    lat, units, _ = form.AddressingInfo()
    lslot, _ = form.PlanInfo()
    assert (lat if numbering == E.NUMBERING_STRUCTURED else lslot) == units == 8  # every block a brick
    op = O.OracleOperator(en, fes.gather_map(), fes.ndofs, order, alpha=c if mass else None, beta=c)
    x = np.random.default_rng(15).uniform(-1, 1, fes.ndofs)
    y = torch.empty(fes.ndofs, dtype=torch.float64, device="cuda")
    form.Mult(dev(x), y)
    assert relerr(host(y), op.mult(x)) <= RTOL
    y2 = torch.empty_like(y)
    form.Mult(dev(x), y2)
    assert torch.equal(y, y2)  # deterministic


@pytest.mark.parametrize("kernel", ["tpe", "wpe"])
@pytest.mark.parametrize("order", [1, 2])
def test_qdata_matches_reference_setup(kernel, order):
    """pa_data == PADiffusionSetup3D / mass setup restated (bilininteg_diffusion_kernels.cpp:243-367)."""
    m = make_mesh("fichera_r1")
    fes, form, op = build_pair(m, order, "bio_a", "bio_b", kernel=KERNELS[kernel])
    qd = form.qdata(E.DIFFUSION)
    qm = form.qdata(E.MASS)[:, 0, :]
    assert relerr(qd, op.D) < 1e-13
    assert relerr(qm, op.M) < 1e-13


@pytest.mark.parametrize("mesh_name,order", [("nonaligned", 2), ("trilinear", 2), ("nonaligned", 4),
                                              ("trilinear", 3)])
def test_jacobian_geometry_path(mesh_name, order):
    """set_jacobians (GeometricFactors layout -- what the reference-side binding passes) gives
    the same operator as element nodes; affine Jacobians (constant per element, checked on
    the device) select the compressed layout; trilinear ones are fitted to the elements'
    trilinear maps (checked at every point) and select the TRILINEAR layout (TRILINEAR_E at
    p >= 3)."""
    m = make_mesh(mesh_name)
    fes = E.H1Space(m, order)
    en = m.element_nodes()
    q1d = O.default_q1d(order)
    _, J, _ = O.geom(en, q1d)
    form = E.BilinearForm(fes, geometry="jacobians")
    form.SetJacobians(dev(J))
    form.AddDomainIntegrator(E.MassIntegrator(E.ConstantCoefficient(3.0)))
    form.AddDomainIntegrator(E.DiffusionIntegrator(E.ConstantCoefficient(0.5)))
    form.Assemble()
    op = O.OracleOperator(en, fes.gather_map(), fes.ndofs, order, alpha=3.0, beta=0.5)
    affine = mesh_name != "trilinear" and AFFINE_ON
    want = (E.QLAYOUT_AFFINE if order <= 2 else E.QLAYOUT_AFFINE_E) if affine else \
        (E.QLAYOUT_TRILINEAR if order <= 2 else E.QLAYOUT_TRILINEAR_E)
    assert form.info()["layout"] == want
    if want in (E.QLAYOUT_TRILINEAR, E.QLAYOUT_TRILINEAR_E):
        assert relerr(form.qdata(E.DIFFUSION), op.D) < 1e-13
    x = np.random.default_rng(5).uniform(-1, 1, fes.ndofs)
    y = torch.empty(fes.ndofs, dtype=torch.float64, device="cuda")
    form.Mult(dev(x), y)
    assert relerr(host(y), op.mult(x)) <= RTOL
    d = torch.empty(fes.ndofs, dtype=torch.float64, device="cuda")
    form.AssembleDiagonal(d)
    assert relerr(host(d), op.diagonal()) < 1e-13


@pytest.mark.parametrize("order", [1, 2, 4])
def test_restriction_and_integrator_pieces(order):
    """ElementRestriction::Mult/MultTranspose and each AddMultPA on E-vectors."""
    m = make_mesh("cart_130")
    fes, form, op = build_pair(m, order, "fn", "fn")
    x = np.random.default_rng(11).uniform(-1, 1, fes.ndofs)
    nd = fes.nd
    xe = torch.empty(fes.ne * nd, dtype=torch.float64, device="cuda")
    form.RestrictionMult(dev(x), xe)
    xe_ref = O.restriction_mult(fes.gather_map(), x)
    assert np.array_equal(host(xe).reshape(fes.ne, nd), xe_ref)
    ye = np.random.default_rng(12).uniform(-1, 1, (fes.ne, nd))
    y = torch.empty(fes.ndofs, dtype=torch.float64, device="cuda")
    form.RestrictionMultTranspose(dev(ye), y)
    assert relerr(host(y), O.restriction_mult_transpose(op.off, op.idx, ye)) < 1e-15
    for kind, ref in ((E.MASS, O.mass_apply(op.B, op.M, xe_ref)),
                      (E.DIFFUSION, O.diffusion_apply(op.B, op.G, op.D, xe_ref))):
        out = torch.zeros(fes.ne * nd, dtype=torch.float64, device="cuda")
        form.IntegratorAddMultPA(kind, dev(xe_ref), out)
        assert relerr(host(out).reshape(fes.ne, nd), ref) <= RTOL


@pytest.mark.parametrize("order", [1, 2, 3, 4])
def test_diagonal_matches_oracle(order):
    m = make_mesh("fichera_r1")
    fes, form, op = build_pair(m, order, "fn", "fn")
    d = torch.empty(fes.ndofs, dtype=torch.float64, device="cuda")
    form.AssembleDiagonal(d)
    assert relerr(host(d), op.diagonal()) < 1e-13


def test_gridfunction_pennes_coefficient():
    """beta = gamma*dt*k(T) with T an H1 grid function: GridFunctionCoefficient projected to
    quadrature points (qfunction.cpp:73-98) then the affine Pennes law."""
    m = make_mesh("fichera_r1")
    order = 2
    fes = E.H1Space(m, order)
    en = m.element_nodes()
    T = temperature(fes.dof_coords())
    scale, slope, tref = 0.5 * 0.1, 0.0012, 37.0
    form = E.BilinearForm(fes)
    form.AddDomainIntegrator(E.MassIntegrator(E.ConstantCoefficient(3.6e6)))
    form.AddDomainIntegrator(E.DiffusionIntegrator(E.AffineGridFunctionCoefficient(dev(T), scale, slope, tref)))
    form.Assemble()
    q1d = O.default_q1d(order)
    Tq = O.interp_evector(T[fes.gather_map()], order, q1d)
    beta = scale * (1.0 + slope * (Tq - tref))
    op = O.OracleOperator(en, fes.gather_map(), fes.ndofs, order, alpha=3.6e6, beta=beta)
    x = np.random.default_rng(9).uniform(-1, 1, fes.ndofs)
    y = torch.empty(fes.ndofs, dtype=torch.float64, device="cuda")
    form.Mult(dev(x), y)
    assert relerr(host(y), op.mult(x)) <= RTOL


@pytest.mark.parametrize("numbering", [E.NUMBERING_STRUCTURED, E.NUMBERING_ENTITY])
@pytest.mark.parametrize("mass", ["quad", "none", "marked"])
def test_coefficient_snapshot(numbering, mass):
    """AFFINE layout with the diffusion coefficient k(T) evaluated in the kernel from a snapshot of
    T's dofs (k_apply_tpe_ts): the operator, its diagonal, the E-vector AddMultPA and the
    reference-layout qdata match the oracle (beta = the affine law of T interpolated at the points,
    as the reference's setup projects it, qfunction.cpp:73-98 / coefficient.cpp:2052-2070), and the
    form without the snapshot; with a MassIntegrator, without one, and with a marked one; the
    snapshot is taken at Assemble (a later change of T does not reach the operator)."""
    n = 8
    if numbering == E.NUMBERING_ENTITY:
        m = E.Mesh.MakeCartesian3D(n, n, n, 1.0, 0.7, 1.3, sfc_ordering=True)
    else:
        m = E.Mesh.MakeCartesian3D(n, n, n, 1.0, 0.7, 1.3)
    if mass == "marked":
        m.SetAttributes(1 + np.arange(m.GetNE()) % 2)
    order = 2
    fes = E.H1Space(m, order, numbering)
    en = m.element_nodes()
    q1d = O.default_q1d(order)
    T = temperature(fes.dof_coords())
    Td = dev(T)
    scale, slope, tref = 0.05, 0.0012, 37.0
    a = alpha_bioheat(O.quad_points(en, q1d))
    eo = "faces" if numbering == E.NUMBERING_ENTITY else "auto"
    forms = {}
    for snap in (True, False):
        f = E.BilinearForm(fes, element_order=eo, coefficient_snapshot=snap)
        if mass != "none":
            mi = E.MassIntegrator(E.QuadratureCoefficient(dev(a.reshape(fes.ne, -1))))
            f.AddDomainIntegrator(mi, [1, 0] if mass == "marked" else None)
        f.AddDomainIntegrator(E.DiffusionIntegrator(E.AffineGridFunctionCoefficient(Td, scale, slope, tref)))
        f.Assemble()
        assert f.info()["layout"] == E.QLAYOUT_AFFINE
        assert f.CoefficientSnapshot() == snap
        forms[snap] = f
    form = forms[True]
    nq = q1d ** 3
    # 8 B per point fewer; the snapshot: one value per dof (regular blocks) or per block lattice slot
    # (lattice-map blocks, 729 per 64 elements)
    snap_bytes = 8 * (fes.ndofs if numbering == E.NUMBERING_STRUCTURED else 729 * ((fes.ne + 63) // 64))
    assert form.qdata_bytes() == forms[False].qdata_bytes() - 8 * fes.ne * nq + snap_bytes
    Tq = O.interp_evector(T[fes.gather_map()], order, q1d)
    beta = scale * (1.0 + slope * (Tq - tref))
    op = O.OracleOperator(en, fes.gather_map(), fes.ndofs, order, alpha=None if mass == "none" else a, beta=beta)
    x = np.random.default_rng(17).uniform(-1, 1, fes.ndofs)
    y = torch.full((fes.ndofs,), float("nan"), dtype=torch.float64, device="cuda")
    y2 = torch.empty_like(y)
    Td.fill_(1.0e3)  # after Assemble: the snapshot (and the reference's qdata) keep the old T
    form.Mult(dev(x), y)
    forms[False].Mult(dev(x), y2)
    want = op.mult_markers(x, m.GetAttributes(), mass_marker=[1, 0]) if mass == "marked" else op.mult(x)
    assert relerr(host(y), want) <= RTOL
    assert relerr(host(y), host(y2)) <= 1e-13
    d = torch.empty_like(y)
    form.AssembleDiagonal(d)
    dwant = op.diagonal_markers(m.GetAttributes(), [("mass", [1, 0]), ("diffusion", None)]) \
        if mass == "marked" else op.diagonal()
    assert relerr(host(d), dwant) < 1e-12
    assert relerr(form.qdata(E.DIFFUSION), op.D) < 1e-12
    if mass == "quad":
        assert relerr(form.qdata(E.MASS)[:, 0, :], op.M) < 1e-13
        xe = np.random.default_rng(18).uniform(-1, 1, (fes.ne, fes.nd))
        ye = torch.zeros(fes.ne * fes.nd, dtype=torch.float64, device="cuda")
        form.IntegratorAddMultPA(E.DIFFUSION, dev(xe), ye)
        assert relerr(host(ye).reshape(fes.ne, fes.nd), O.diffusion_apply(op.B, op.G, op.D, xe)) <= RTOL
    # the diagonal is kept per assembly: a second request returns the same values; after T changes
    # and the form is re-assembled it follows the new T (not the kept copy)
    d2 = torch.empty_like(y)
    form.AssembleDiagonal(d2)
    assert torch.equal(d, d2)
    T2 = T + 5.0 * np.sin(3.0 * fes.dof_coords()[:, 0])
    Td.copy_(dev(T2))
    form.Assemble()
    form.AssembleDiagonal(d2)
    beta2 = scale * (1.0 + slope * (O.interp_evector(T2[fes.gather_map()], order, q1d) - tref))
    op2 = O.OracleOperator(en, fes.gather_map(), fes.ndofs, order, alpha=None if mass == "none" else a, beta=beta2)
    dwant2 = op2.diagonal_markers(m.GetAttributes(), [("mass", [1, 0]), ("diffusion", None)]) \
        if mass == "marked" else op2.diagonal()
    assert relerr(host(d2), dwant2) < 1e-12 and relerr(host(d2), dwant) > 1e-9  # (the mass term dominates)
    # a marked diffusion integrator keeps the stored W beta
    f3 = E.BilinearForm(fes, element_order=eo)
    f3.AddDomainIntegrator(E.DiffusionIntegrator(E.AffineGridFunctionCoefficient(dev(T), scale, slope, tref)), [1, 1])
    m.SetAttributes(np.ones(m.GetNE(), dtype=int))
    f3.Assemble()
    assert not f3.CoefficientSnapshot()


@pytest.mark.parametrize("numbering", [E.NUMBERING_STRUCTURED, E.NUMBERING_ENTITY])
@pytest.mark.parametrize("with_ess", [True, False])
def test_pcg_energy_folded_den(numbering, with_ess):
    """CGSolver's den = (A d, d) folded into the snapshot kernel's element energies (sum_e d~_e . A_e d~_e
    with the ess entries zeroed, plus sum_ess d_i^2 for the DIAG_ONE rows; PAForm::mult_energy): the
    device PCG on a snapshot form takes that path (EnergyParts() > 0) and returns CGSolver's iterates --
    x after a fixed 6 iterations and a converging solve's stopping iteration and x -- against the oracle
    (solvers.cpp:869-1004), with and without essential dofs, in both numberings."""
    n, order = 8, 2
    sfc = numbering == E.NUMBERING_ENTITY
    m = E.Mesh.MakeCartesian3D(n, n, n, 1.0, 0.7, 1.3, sfc_ordering=sfc)
    fes = E.H1Space(m, order, numbering)
    en = m.element_nodes()
    q1d = O.default_q1d(order)
    T = temperature(fes.dof_coords())
    scale, slope, tref = 0.05, 0.0012, 37.0
    a = alpha_bioheat(O.quad_points(en, q1d)) / 3.6e6
    form = E.BilinearForm(fes, element_order="faces" if sfc else "auto")
    form.AddDomainIntegrator(E.MassIntegrator(E.QuadratureCoefficient(dev(a.reshape(fes.ne, -1)))))
    form.AddDomainIntegrator(E.DiffusionIntegrator(E.AffineGridFunctionCoefficient(dev(T), scale, slope, tref)))
    form.Assemble()
    assert form.CoefficientSnapshot() and form.EnergyParts() == ((fes.ne + 63) // 64 + 3) // 4
    Tq = O.interp_evector(T[fes.gather_map()], order, q1d)
    op = O.OracleOperator(en, fes.gather_map(), fes.ndofs, order, alpha=a, beta=scale * (1.0 + slope * (Tq - tref)))
    ess = fes.boundary_dofs() if with_ess else np.zeros(0, np.int32)
    esst = dev(ess, torch.int32) if ess.size else None
    b = np.random.default_rng(23).uniform(-1, 1, fes.ndofs)
    x = torch.empty(fes.ndofs, dtype=torch.float64, device="cuda")
    it, nrm = form.PCG(dev(b), x, ess=esst, rel_tol=0.0, max_iter=6, jacobi=True)
    xr, itr, nr = op.pcg(b, ess, rel_tol=0.0, max_iter=6, jacobi=True)
    assert it == itr == 6 and relerr(host(x), xr) < 1e-11 and nrm == pytest.approx(nr, rel=1e-9)
    it, nrm = form.PCG(dev(b), x, ess=esst, rel_tol=1e-12, max_iter=2000, jacobi=True)
    xr, itr, nr = op.pcg(b, ess, rel_tol=1e-12, max_iter=2000, jacobi=True)
    assert abs(it - itr) <= 2 and E.pcg_last_converged() and relerr(host(x), xr) < 1e-9


@pytest.mark.parametrize("snap", [True, False])
def test_marker_diagonal_keeps_assemble_time_state(snap):
    """Diffusion k(T) added first, then a MassIntegrator(perfusion(T)) restricted to attribute 1; T
    changes after Assemble.  AssembleDiagonal follows the reference's shared-localY rule
    (bilinearform_ext.cpp:370-411) on the Assemble-time coefficients (the reference builds it from
    the pa_data stored at Assemble), and leaves no element mask behind: the Mult, the diffusion
    qdata and its E-vector AddMultPA afterwards still describe the unmasked diffusion."""
    import bioheat as BH
    n, order = 8, 2
    m = E.Mesh.MakeCartesian3D(n, n, n, 1.0, 0.7, 1.3)
    m.SetAttributes(1 + np.arange(m.GetNE()) % 2)
    fes = E.H1Space(m, order, E.NUMBERING_STRUCTURED)
    en = m.element_nodes()
    q1d = O.default_q1d(order)
    T = temperature(fes.dof_coords())
    Td = dev(T)
    par = (3.6e6, 0.05 * 3.6e3, 6.4e-3, 0.02, 37.0, 1e300)
    ks, kslope, ktref = 0.05, 0.0012, 37.0
    f = E.BilinearForm(fes, coefficient_snapshot=snap)
    f.AddDomainIntegrator(E.DiffusionIntegrator(E.AffineGridFunctionCoefficient(Td, ks, kslope, ktref)))
    f.AddDomainIntegrator(E.MassIntegrator(E.PerfusionCoefficient(Td, *par)), [1, 0])
    f.Assemble()
    assert f.CoefficientSnapshot() == snap
    Tq = BH.temperature_at_quadrature(T, fes.gather_map(), order, q1d)
    op = O.OracleOperator(en, fes.gather_map(), fes.ndofs, order, alpha=BH.perfusion_law(Tq, *par),
                          beta=BH.affine_law(Tq, ks, kslope, ktref))
    Td.fill_(1.0e3)  # after Assemble: neither the operator nor its diagonal may see it
    attr = m.GetAttributes()
    d = torch.full((fes.ndofs,), float("nan"), dtype=torch.float64, device="cuda")
    f.AssembleDiagonal(d)
    assert relerr(host(d), op.diagonal_markers(attr, [("diffusion", None), ("mass", [1, 0])])) < 1e-12
    x = np.random.default_rng(5).uniform(-1, 1, fes.ndofs)
    y = torch.full_like(d, float("nan"))
    f.Mult(dev(x), y)
    assert relerr(host(y), op.mult_markers(x, attr, mass_marker=[1, 0])) <= RTOL
    assert relerr(f.qdata(E.DIFFUSION), op.D) < 1e-12
    xe = np.random.default_rng(6).uniform(-1, 1, (fes.ne, fes.nd))
    ye = torch.zeros(fes.ne * fes.nd, dtype=torch.float64, device="cuda")
    f.IntegratorAddMultPA(E.DIFFUSION, dev(xe), ye)
    assert relerr(host(ye).reshape(fes.ne, fes.nd), O.diffusion_apply(op.B, op.G, op.D, xe)) <= RTOL
    d2 = torch.full_like(d, float("nan"))
    f.AssembleDiagonal(d2)
    assert torch.equal(d, d2)


@pytest.mark.parametrize("name,order,q1d", [("fichera-q2.mesh", 2, 4), ("fichera-q2.mesh", 2, 5), ("fichera-q2.mesh", 3, 5),
                                         ("fichera-q2.mesh", 3, 6), ("fichera-q3.mesh", 3, 5), ("fichera-q3.mesh", 3, 6),
                                         ("fichera-q3.mesh", 4, 6)])
def test_curved_mesh_jacobians(tmp_path, name, order, q1d):
    """A curved (high-order-node) mesh through the drop-in boundary: the reference's data/fichera-q2.mesh
    (H1_3D_P2 nodes) and data/fichera-q3.mesh (the legacy Cubic collection; the curved fichera meshes of
    test_assembly_levels.cpp:230,260 and test_pa_kernels.cpp:647, the orders >= the map's so that the
    linear function below is in the space) handed over as GeometricFactors::JACOBIANS at the rule's points
    (ecm2_pa_form_set_jacobians, as INTEGRATION.md's binding passes them).  No trilinear map produces
    them, so the form keeps the per-point layout; Q1D = p + 3 is the rule a quadratic mesh's
    MassIntegrator asks for (GetRule adds Trans.OrderW(), bilininteg.cpp:1450-1462).  Mult and diagonal
    against the oracle on the same Jacobians, and the geometry-independent identities through the HIP
    path (1^T M 1 = sum W det J, K 1 = 0, x^T K x = |g|^2 sum W det J for the linear x = g . X)."""
    mesh, fes, J, X = H.curved_fichera(tmp_path, order, q1d, name)
    gm = fes.gather_map()
    en = mesh.element_nodes()
    P = O.quad_points(en, q1d)           # (coefficient sample points: any smooth per-point values)
    a, b = alpha_bioheat(P), coeff_function(P)
    form = E.BilinearForm(fes, q1d=q1d, geometry="jacobians")
    form.SetJacobians(dev(J))
    form.AddDomainIntegrator(E.MassIntegrator(E.QuadratureCoefficient(dev(a.reshape(fes.ne, -1)))))
    form.AddDomainIntegrator(E.DiffusionIntegrator(E.QuadratureCoefficient(dev(b.reshape(fes.ne, -1)))))
    form.Assemble()
    assert form.info()["layout"] not in (E.QLAYOUT_AFFINE, E.QLAYOUT_TRILINEAR, E.QLAYOUT_AFFINE_E,
                                         E.QLAYOUT_TRILINEAR_E)   # curved: the per-point layout
    op = O.OracleOperator.from_jacobians(J, gm, fes.ndofs, order, alpha=a, beta=b, q1d=q1d)
    x = np.random.default_rng(order * 10 + q1d).uniform(-1, 1, fes.ndofs)
    y = torch.full((fes.ndofs,), float("nan"), dtype=torch.float64, device="cuda")
    form.Mult(dev(x), y)
    assert relerr(host(y), op.mult(x)) <= RTOL
    d = torch.full_like(y, float("nan"))
    form.AssembleDiagonal(d)
    assert relerr(host(d), op.diagonal()) <= RTOL
    vol = float((np.linalg.det(np.transpose(J, (0, 3, 2, 1))) * O.cube_weights(q1d)).sum())
    for kind in ("mass", "diffusion"):
        f = E.BilinearForm(fes, q1d=q1d, geometry="jacobians")
        f.SetJacobians(dev(J))
        f.AddDomainIntegrator(E.MassIntegrator() if kind == "mass" else E.DiffusionIntegrator())
        f.Assemble()
        one = torch.ones(fes.ndofs, dtype=torch.float64, device="cuda")
        yy = torch.empty_like(one)
        f.Mult(one, yy)
        if kind == "mass":
            assert abs(float(yy.sum()) - vol) < 1e-12 * vol
        else:
            assert float(yy.abs().max()) < 1e-12
            g = np.array([0.3, -1.1, 0.7])
            xg = dev(X @ g)
            f.Mult(xg, yy)
            assert abs(float(torch.dot(xg, yy)) - (g @ g) * vol) < 1e-11 * (g @ g) * vol


@pytest.mark.parametrize("order,q1d", [(1, 3), (2, 3), (2, 5), (3, 4), (4, 5), (4, 7)])
@pytest.mark.parametrize("geometry", ["nodes", "jacobians"])
def test_integration_rule_q1d(order, q1d, geometry):
    """The rule the integrator asks for, passed through the ABI as q1d (ecm2_pa_form_create): MFEM's
    AssemblePA takes IntRule ? IntRule : GetRule(el, el[, T]) (bilininteg_diffusion_pa.cpp:97,
    bilininteg_mass_pa.cpp:34), which differs from the default Q1D = p + 2 for a user rule or a
    high-order mesh (MassIntegrator::GetRule adds Trans.OrderW(), bilininteg.cpp:1450-1462; a
    quadratic mesh gives Q1D = p + 3).  Mult and diagonal on fichera r1 (the reference's numbering,
    non-lattice blocks) against the oracle on the same Gauss-Legendre rule, geometry as corners or
    as MFEM Jacobians at that rule's points."""
    m = make_mesh("fichera_r1")
    fes = E.H1Space(m, order)
    en = m.element_nodes()
    P = O.quad_points(en, q1d)
    a, b = alpha_bioheat(P), coeff_function(P)
    form = E.BilinearForm(fes, q1d=q1d, geometry=geometry)
    assert form.info()["q1d"] == q1d
    if geometry == "jacobians":
        form.SetJacobians(m.jacobians(q1d))
    form.AddDomainIntegrator(E.MassIntegrator(E.QuadratureCoefficient(dev(a.reshape(fes.ne, -1)))))
    form.AddDomainIntegrator(E.DiffusionIntegrator(E.QuadratureCoefficient(dev(b.reshape(fes.ne, -1)))))
    form.Assemble()
    op = O.OracleOperator(en, fes.gather_map(), fes.ndofs, order, alpha=a, beta=b, q1d=q1d)
    x = np.random.default_rng(q1d).uniform(-1, 1, fes.ndofs)
    y = torch.full((fes.ndofs,), float("nan"), dtype=torch.float64, device="cuda")
    form.Mult(dev(x), y)
    assert relerr(host(y), op.mult(x)) <= RTOL
    d = torch.full_like(y, float("nan"))
    form.AssembleDiagonal(d)
    assert relerr(host(d), op.diagonal()) <= RTOL
    # a wrong-sized coefficient (the default rule's points) is refused before it reaches the GPU
    if q1d != order + 2:
        f2 = E.BilinearForm(fes, q1d=q1d)
        Pd = O.quad_points(en, order + 2)
        with pytest.raises(E.ECM2Error):
            f2.AddDomainIntegrator(E.MassIntegrator(E.QuadratureCoefficient(dev(alpha_bioheat(Pd).reshape(fes.ne, -1)))))


@pytest.mark.parametrize("jacobi", [True, False])
def test_pcg_matches_oracle(jacobi):
    m = make_mesh("fichera_r1")
    order = 2
    fes, form, op = build_pair(m, order, 1.0, "fn")
    ess = fes.boundary_dofs()
    b = np.random.default_rng(4).uniform(-1, 1, fes.ndofs)
    x = torch.empty(fes.ndofs, dtype=torch.float64, device="cuda")
    it, nrm = form.PCG(dev(b), x, ess=dev(ess, torch.int32), rel_tol=1e-12, max_iter=2000, jacobi=jacobi)
    xr, itr, _ = op.pcg(b, ess, rel_tol=1e-12, max_iter=2000, jacobi=jacobi)
    assert abs(it - itr) <= 2
    assert relerr(host(x), xr) < 1e-9


@pytest.mark.parametrize("max_iter", [1, 2, 3, 4, 5, 8])
def test_pcg_device_loop_stops_like_cgsolver(max_iter):
    """The device-driven PCG loop (the stopping test in a kernel, iterations enqueued up to
    kPcgAhead ahead, later vector kernels no-ops once stopped) returns CGSolver's iterate: after
    max_iter iterations (fewer and more than the run-ahead window) x equals the oracle's after the
    same count, and a converging solve stops at the oracle's iteration (solvers.cpp:930-1000)."""
    m = make_mesh("fichera_r1")
    fes, form, op = build_pair(m, 2, 1.0, "fn")
    ess = fes.boundary_dofs()
    b = np.random.default_rng(6).uniform(-1, 1, fes.ndofs)
    x = torch.empty(fes.ndofs, dtype=torch.float64, device="cuda")
    it, nrm = form.PCG(dev(b), x, ess=dev(ess, torch.int32), rel_tol=1e-30, max_iter=max_iter, jacobi=True)
    xr, itr, nr = op.pcg(b, ess, rel_tol=1e-30, max_iter=max_iter, jacobi=True)
    assert it == itr == max_iter
    assert relerr(host(x), xr) < 1e-11 and nrm == pytest.approx(nr, rel=1e-9)
    # converging at a loose tolerance: the same stopping iteration, then every later kernel idle
    it, nrm = form.PCG(dev(b), x, ess=dev(ess, torch.int32), rel_tol=1e-3, max_iter=500, jacobi=True)
    xr, itr, nr = op.pcg(b, ess, rel_tol=1e-3, max_iter=500, jacobi=True)
    assert it == itr and relerr(host(x), xr) < 1e-11


@pytest.mark.parametrize("case", ["spd", "indefinite_mid", "indefinite_first", "negative_start", "zero_operator",
                                  "nan_rhs"])
def test_pcg_device_stops_like_cgsolver_indefinite(case):
    """CGSolver's other stops (solvers.cpp:893-1004) in the device-driven loop, against
    the oracle (pinned by tests/test_oracle_pins.py::test_pcg_oracle_stops_like_cgsolver): a mass
    coefficient of -amp on x > 0.7 makes the Jacobi diagonal indefinite, so (B r, r) < 0 stops the
    loop not converged in the loop (final_iter = i) or before it (final_iter 0, final_norm = nom); a
    zero operator without a preconditioner stops at (A d, d) == 0; a NaN right-hand side is
    MFEM_VERIFY's abort, ECM2_ERR_NUMERIC."""
    m = E.Mesh.MakeCartesian3D(4, 4, 4)
    m.set_vertices(nonaligned(m.vertices()))
    fes = E.H1Space(m, 2)
    en = m.element_nodes()
    P = O.quad_points(en, O.default_q1d(2))
    amp, beta, jacobi, expect = {"spd": (-1.0, 0.5, True, 1), "indefinite_mid": (30.0, 0.05, True, 3),
                                 "indefinite_first": (40.0, 0.05, True, 3), "negative_start": (60.0, 0.05, True, 3),
                                 "zero_operator": (0.0, 0.0, False, 4), "nan_rhs": (-1.0, 0.5, True, 5)}[case]
    alpha = np.where(P[..., 0] > 0.7, -amp, 1.0) if case != "zero_operator" else np.zeros(P.shape[:-1])
    form = E.BilinearForm(fes)
    form.AddDomainIntegrator(E.MassIntegrator(E.QuadratureCoefficient(dev(alpha.reshape(fes.ne, -1)))))
    form.AddDomainIntegrator(E.DiffusionIntegrator(E.ConstantCoefficient(beta)))
    form.Assemble()
    op = O.OracleOperator(en, fes.gather_map(), fes.ndofs, 2, alpha=alpha, beta=beta)
    X = fes.dof_coords()
    ess = np.nonzero(np.isclose(X[:, 0], 0))[0].astype(np.int32) if case != "zero_operator" else np.zeros(0, np.int32)
    b = np.random.default_rng(0).uniform(-1, 1, fes.ndofs)
    if case == "nan_rhs":
        b[5] = np.nan
    x = torch.empty(fes.ndofs, dtype=torch.float64, device="cuda")
    esst = dev(ess, torch.int32) if ess.size else None
    xr, itr, nr = op.pcg(b, ess, rel_tol=1e-10, max_iter=300, jacobi=jacobi)
    assert op.last_pcg_status == expect
    if case == "nan_rhs":
        with pytest.raises(E.ECM2Error) as ei:
            form.PCG(dev(b), x, ess=esst, rel_tol=1e-10, max_iter=300, jacobi=jacobi)
        assert ei.value.code == 8  # ECM2_ERR_NUMERIC
        return
    it, nrm = form.PCG(dev(b), x, ess=esst, rel_tol=1e-10, max_iter=300, jacobi=jacobi)
    assert it == itr
    assert E.pcg_last_converged() == (expect == 1)
    if case == "indefinite_mid":
        assert it > 1
    if it > 0:
        assert relerr(host(x), xr) < 1e-9
    if case == "negative_start":
        assert it == 0 and nrm < 0 and nrm == pytest.approx(nr, rel=1e-12)


def test_golden_vectors():
    g = np.load(f"{GOLDEN}/oracle_golden.npz")
    for order in (1, 2, 3):
        m = E.Mesh.MakeCartesian3D(2, 2, 2)
        m.set_vertices(nonaligned(m.vertices()))
        fes = E.H1Space(m, order, E.NUMBERING_STRUCTURED)
        _, form, _ = build_pair(m, order, "fn", "fn", numbering=E.NUMBERING_STRUCTURED)
        y = torch.empty(fes.ndofs, dtype=torch.float64, device="cuda")
        form.Mult(dev(g[f"p{order}_x"]), y)
        assert relerr(host(y), g[f"p{order}_y"]) <= RTOL
        d = torch.empty(fes.ndofs, dtype=torch.float64, device="cuda")
        form.AssembleDiagonal(d)
        assert relerr(host(d), g[f"p{order}_diag"]) < 1e-13


def test_edge_cases():
    # single element, p = 2 and p = 4
    for order in (2, 4):
        m = E.Mesh.MakeCartesian3D(1, 1, 1)
        fes, form, op = build_pair(m, order, "fn", "fn")
        x = np.random.default_rng(1).uniform(-1, 1, fes.ndofs)
        y = torch.empty(fes.ndofs, dtype=torch.float64, device="cuda")
        form.Mult(dev(x), y)
        assert relerr(host(y), op.mult(x)) <= RTOL
    # zero input -> zero output; Mult before Assemble raises
    m = make_mesh("nonaligned")
    fes = E.H1Space(m, 2)
    f2 = E.BilinearForm(fes)
    f2.AddDomainIntegrator(E.MassIntegrator())
    y = torch.empty(fes.ndofs, dtype=torch.float64, device="cuda")
    with pytest.raises(E.ECM2Error):
        f2.Mult(torch.zeros_like(y), y)
    f2.Assemble()
    f2.Mult(torch.zeros_like(y), y)
    assert float(y.abs().max()) == 0.0
    # a dof referenced by no element (extra unused dof) -> 0, like ElementRestriction::MultTranspose
    gm = fes.gather_map()
    f3 = E.load_library()
    import ctypes
    h = ctypes.c_void_p()
    E._check(f3.ecm2_pa_form_create(fes.ne, 2, fes.ndofs + 5, ctypes.c_void_p(gm.ctypes.data), 0, ctypes.byref(h)))
    en = m.element_nodes()
    E._check(f3.ecm2_pa_form_set_element_nodes(h, ctypes.c_void_p(en.ctypes.data)))
    one = (ctypes.c_double * 1)(1.0)
    E._check(f3.ecm2_pa_form_add_integrator(h, E.MASS, E.COEFF_CONSTANT, ctypes.cast(one, ctypes.c_void_p), None))
    E._check(f3.ecm2_pa_form_assemble(h, E._stream()))
    xx = torch.ones(fes.ndofs + 5, dtype=torch.float64, device="cuda")
    yy = torch.full_like(xx, 7.0)
    E._check(f3.ecm2_pa_form_mult(h, E._dev_ptr(xx), E._dev_ptr(yy), E._stream()))
    assert np.all(host(yy)[-5:] == 0.0)
    f3.ecm2_pa_form_destroy(h)
    # invalid gather map is rejected
    bad = gm.copy()
    bad[0, 0] = fes.ndofs + 100
    with pytest.raises(E.ECM2Error):
        E._check(f3.ecm2_pa_form_create(fes.ne, 2, fes.ndofs, ctypes.c_void_p(bad.ctypes.data), 0, ctypes.byref(h)))


@pytest.mark.parametrize("numbering", [E.NUMBERING_STRUCTURED, E.NUMBERING_ENTITY])
def test_full_size_c2(numbering):
    """BASELINE config[1] (inline-hex refined to ~1M DoF, p = 2) at full size: direct oracle
    parity, plus size-independent properties (linearity, symmetry, 1^T M 1 = int alpha)."""
    n = 50
    m = E.Mesh.MakeCartesian3D(n, n, n)
    fes, form, op = build_pair(m, 2, "bio_a", "bio_b", numbering=numbering)
    assert fes.ndofs == 1030301
    rng = np.random.default_rng(21)
    x1 = rng.uniform(-1, 1, fes.ndofs)
    x2 = rng.uniform(-1, 1, fes.ndofs)
    y1 = torch.empty(fes.ndofs, dtype=torch.float64, device="cuda")
    y2 = torch.empty_like(y1)
    y3 = torch.empty_like(y1)
    form.Mult(dev(x1), y1)
    form.Mult(dev(x2), y2)
    form.Mult(dev(2.0 * x1 - 3.0 * x2), y3)
    h1, h2, h3 = host(y1), host(y2), host(y3)
    assert relerr(h1, op.mult(x1)) <= RTOL
    assert relerr(h3, 2.0 * h1 - 3.0 * h2) <= 1e-12
    assert abs(x2 @ h1 - x1 @ h2) <= 1e-12 * abs(x2) @ np.abs(h1)


def test_full_size_c4_tpe():
    """configs[3] size (Cartesian 108^3, p = 2, 10.2M DoF) on one GPU against the oracle."""
    n = 108
    m = E.Mesh.MakeCartesian3D(n, n, n)
    fes, form, op = build_pair(m, 2, "bio_a", "bio_b", numbering=E.NUMBERING_STRUCTURED)
    assert fes.ndofs == 10218313
    assert form.info()["layout"] == (E.QLAYOUT_AFFINE if AFFINE_ON else E.QLAYOUT_BLOCKED)  # i/108 lattice: affine
    x = np.random.default_rng(22).uniform(-1, 1, fes.ndofs)
    y = torch.empty(fes.ndofs, dtype=torch.float64, device="cuda")
    form.Mult(dev(x), y)
    assert relerr(host(y), op.mult(x)) <= RTOL


@pytest.mark.parametrize("mesh_kind", ["affine", "trilinear", "trilinear_jacobians"])
def test_full_size_c4_reference_numbering(mesh_kind):
    """configs[3] size with the reference's own numbering -- MakeCartesian3D's space-filling-curve
    element order and FiniteElementSpace's entity dofs, the element order derived by the form from
    the map (what a drop-in binding gets; bench.py's entity_numbering sub-object) -- and, second
    case, the same mesh with its interior vertices moved (TRILINEAR layout): against the oracle,
    plus the diagonal. Third case: the full drop-in configuration (bench.py's drop_in sub-object)
    -- the same perturbed mesh, but the geometry handed over as J at the quadrature points
    (SetJacobians, what GeometricFactors gives the reference's PA setup), fitted to TRILINEAR."""
    n = 108
    m = E.Mesh.MakeCartesian3D(n, n, n, sfc_ordering=True)
    if mesh_kind.startswith("trilinear"):
        V = m.vertices()
        h = 1.0 / n
        inner = np.all((V > 0.5 * h) & (V < 1.0 - 0.5 * h), axis=1)
        V[inner] += 0.15 * h * np.random.default_rng(7).uniform(-1, 1, (int(inner.sum()), 3))
        m.set_vertices(V)
    geo = "jacobians" if mesh_kind == "trilinear_jacobians" else "nodes"
    fes, form, op = build_pair(m, 2, "bio_a", "bio_b", numbering=E.NUMBERING_ENTITY, element_order="faces",
                               geometry=geo)
    assert fes.ndofs == 10218313
    assert form.info()["layout"] == (E.QLAYOUT_AFFINE if mesh_kind == "affine" else E.QLAYOUT_TRILINEAR)
    lslot, _ = form.PlanInfo()
    assert lslot == (n // 4) ** 3  # every 4x4x4 brick reads a lattice map and keeps face-grouped slots
    x = np.random.default_rng(23).uniform(-1, 1, fes.ndofs)
    y = torch.empty(fes.ndofs, dtype=torch.float64, device="cuda")
    form.Mult(dev(x), y)
    assert relerr(host(y), op.mult(x)) <= RTOL
    d = torch.empty_like(y)
    form.AssembleDiagonal(d)
    assert relerr(host(d), op.diagonal()) < 1e-13


@pytest.mark.parametrize("element_order", ["native", "brick", "morton"])
@pytest.mark.parametrize("order", [1, 2])
def test_element_orders_same_operator(element_order, order):
    """The blocked layout's element permutation and in-wave face assembly are invisible:
    every order gives the oracle's y (cart_bricks has complete bricks and leftovers)."""
    m = make_mesh("cart_bricks")
    fes, form, op = build_pair(m, order, "fn", "fn", element_order=element_order)
    x = np.random.default_rng(31).uniform(-1, 1, fes.ndofs)
    y = torch.empty(fes.ndofs, dtype=torch.float64, device="cuda")
    form.Mult(dev(x), y)
    assert relerr(host(y), op.mult(x)) <= RTOL
    qd = form.qdata(E.DIFFUSION)
    assert relerr(qd, op.D) < 1e-13
    d = torch.empty(fes.ndofs, dtype=torch.float64, device="cuda")
    form.AssembleDiagonal(d)
    assert relerr(host(d), op.diagonal()) < 1e-13


@pytest.mark.parametrize("mesh_name", ["nonaligned", "fichera_r1", "cart_bricks", "cart_130"])
@pytest.mark.parametrize("element_order", ["native", "brick", "morton"])
@pytest.mark.parametrize("order", [1, 2])
def test_scatter_modes(mesh_name, element_order, order):
    """Partial-slot scatter (default) and atomic scatter both give the oracle's y; the
    partial scatter overwrites every entry (y pre-filled with NaN) and is bitwise
    reproducible."""
    m = make_mesh(mesh_name)
    if element_order == "brick" and mesh_name == "fichera_r1":
        pytest.skip("brick order needs a Cartesian mesh")
    x = np.random.default_rng(41).uniform(-1, 1, make_fes_ndofs(m, order))
    ys = {}
    for scatter in ("partials", "atomic"):
        fes, form, op = build_pair(m, order, "fn", "fn", element_order=element_order, scatter=scatter)
        y = torch.full((fes.ndofs,), float("nan"), dtype=torch.float64, device="cuda")
        form.Mult(dev(x), y)
        assert relerr(host(y), op.mult(x)) <= RTOL
        ys[scatter] = host(y)
        if scatter == "partials":
            n_sh, n_slots = form.ScatterInfo()
            assert 0 <= n_sh <= fes.ndofs and n_slots >= 2 * n_sh - fes.ndofs
            for _ in range(3):
                y2 = torch.full_like(y, float("nan"))
                form.Mult(dev(x), y2)
                assert torch.equal(y, y2)
    assert relerr(ys["partials"], ys["atomic"]) <= RTOL


def make_fes_ndofs(m, order):
    return E.H1Space(m, order).ndofs


def test_full_size_c2_deterministic():
    """C2 size: the default fused Mult is bitwise reproducible and matches the atomic scatter."""
    n = 50
    m = E.Mesh.MakeCartesian3D(n, n, n)
    fes = E.H1Space(m, 2, E.NUMBERING_STRUCTURED)
    x = dev(np.random.default_rng(23).uniform(-1, 1, fes.ndofs))
    out = {}
    for scatter in ("partials", "atomic"):
        form = E.BilinearForm(fes, scatter=scatter)
        form.AddDomainIntegrator(E.MassIntegrator(E.ConstantCoefficient(2.0)))
        form.AddDomainIntegrator(E.DiffusionIntegrator(E.ConstantCoefficient(0.3)))
        form.Assemble()
        y = torch.full((fes.ndofs,), float("nan"), dtype=torch.float64, device="cuda")
        form.Mult(x, y)
        out[scatter] = y
        if scatter == "partials":
            y2 = torch.empty_like(y)
            form.Mult(x, y2)
            assert torch.equal(y, y2)
    assert relerr(host(out["partials"]), host(out["atomic"])) <= RTOL


@pytest.mark.parametrize("mesh_name", ["inline_hex", "cart_bricks", "nonaligned", "fichera_r1", "cart_130"])
@pytest.mark.parametrize("order", [3, 4, 5, 6])
def test_line_bricks(mesh_name, order):
    """p >= 3 brick kernel (2 x 2 x 1 and 2 x 2 x 2 workgroups, LDS lattice assembly) and the
    per-element line kernel it falls back to: each matches the oracle, overwrites every y
    entry (NaN prefill), is bitwise reproducible, and the brick modes agree."""
    m = make_mesh(mesh_name)
    ys = {}
    for bz in (0, 1, 2):
        fes = E.H1Space(m, order)
        form = E.BilinearForm(fes, kernel=E.KERNEL_LINE, bricks=bz)
        en = m.element_nodes()
        P = O.quad_points(en, O.default_q1d(order))
        a, b = alpha_bioheat(P), coeff_function(P)
        form.AddDomainIntegrator(E.MassIntegrator(E.QuadratureCoefficient(dev(a.reshape(fes.ne, -1)))))
        form.AddDomainIntegrator(E.DiffusionIntegrator(E.QuadratureCoefficient(dev(b.reshape(fes.ne, -1)))))
        form.Assemble()
        nb, depth = form.BrickInfo()
        if bz == 0:
            assert nb == 0
        elif mesh_name in ("inline_hex", "cart_bricks"):
            assert nb > 0 and depth == (bz if order < 6 else 1)  # 2 x 2 x 2 bricks exceed LDS at p = 6
        x = np.random.default_rng(order).uniform(-1, 1, fes.ndofs)
        y = torch.full((fes.ndofs,), float("nan"), dtype=torch.float64, device="cuda")
        form.Mult(dev(x), y)
        op = O.OracleOperator(en, fes.gather_map(), fes.ndofs, order, alpha=a, beta=b)
        assert relerr(host(y), op.mult(x)) <= RTOL, (bz, nb)
        y2 = torch.full_like(y, float("nan"))
        form.Mult(dev(x), y2)
        assert torch.equal(y, y2)
        ys[bz] = host(y)
    assert relerr(ys[1], ys[0]) <= RTOL and relerr(ys[2], ys[0]) <= RTOL


def test_full_size_c5_bricks():
    """C5-shaped (order 4, Cartesian) at a size the oracle finishes quickly: bricks cover
    every element of an even mesh; the Mult matches the oracle and the per-element kernel."""
    m = E.Mesh.MakeCartesian3D(12, 10, 8)
    fes = E.H1Space(m, 4, E.NUMBERING_STRUCTURED)
    en = m.element_nodes()
    P = O.quad_points(en, 6)
    a, b = alpha_bioheat(P), k_of_T(temperature(P))
    x = np.random.default_rng(5).uniform(-1, 1, fes.ndofs)
    out = {}
    for bz in (0, 1, 2):
        form = E.BilinearForm(fes, bricks=bz)
        form.AddDomainIntegrator(E.MassIntegrator(E.QuadratureCoefficient(dev(a.reshape(fes.ne, -1)))))
        form.AddDomainIntegrator(E.DiffusionIntegrator(E.QuadratureCoefficient(dev(b.reshape(fes.ne, -1)))))
        form.Assemble()
        if bz:
            assert form.BrickInfo() == (fes.ne // (4 * bz), bz)
        y = torch.full((fes.ndofs,), float("nan"), dtype=torch.float64, device="cuda")
        form.Mult(dev(x), y)
        out[bz] = host(y)
    ref = O.OracleOperator(en, fes.gather_map(), fes.ndofs, 4, alpha=a, beta=b).mult(x)
    for bz in out:
        assert relerr(out[bz], ref) <= RTOL, bz


@pytest.mark.parametrize("order", [3, 4, 5])
@pytest.mark.parametrize("geometry", ["nodes", "jacobians"])
def test_trilinear_e_bricks(order, geometry):
    """TRILINEAR_E at p >= 3 (a non-affine mesh: the element's trilinear-map coefficients + one
    (W beta / det J, W alpha det J) pair per point; the brick kernel's z stage evaluates J and
    adj(J) at its points): 2 x 2 x 1 and 2 x 2 x 2 bricks and the per-element line kernel against
    the oracle (bitwise reproducible), from corners and from the reference binding's Jacobians,
    plus the diagonal and the reference-layout qdata."""
    m = E.Mesh.MakeCartesian3D(6, 4, 4)
    V = m.vertices()
    inner = np.all((V > 1e-9) & (V < np.array([1.0, 1.0, 1.0]) - 1e-9), axis=1)
    V[inner] += 0.04 * np.random.default_rng(12).uniform(-1, 1, (int(inner.sum()), 3))
    m.set_vertices(V)
    fes = E.H1Space(m, order)
    en = m.element_nodes()
    q1d = O.default_q1d(order)
    P = O.quad_points(en, q1d)
    a, b = alpha_bioheat(P), coeff_function(P)
    op = O.OracleOperator(en, fes.gather_map(), fes.ndofs, order, alpha=a, beta=b)
    x = np.random.default_rng(order).uniform(-1, 1, fes.ndofs)
    for bz in (0, 1, 2):
        form = E.BilinearForm(fes, kernel=E.KERNEL_LINE, bricks=bz, geometry=geometry)
        if geometry == "jacobians":
            form.SetJacobians(m.jacobians(q1d))
        form.AddDomainIntegrator(E.MassIntegrator(E.QuadratureCoefficient(dev(a.reshape(fes.ne, -1)))))
        form.AddDomainIntegrator(E.DiffusionIntegrator(E.QuadratureCoefficient(dev(b.reshape(fes.ne, -1)))))
        form.Assemble()
        assert form.info()["layout"] == E.QLAYOUT_TRILINEAR_E
        nb, depth = form.BrickInfo()
        assert (nb > 0) == (bz > 0)
        y = torch.full((fes.ndofs,), float("nan"), dtype=torch.float64, device="cuda")
        form.Mult(dev(x), y)
        assert relerr(host(y), op.mult(x)) <= RTOL, (bz, nb, depth)
        y2 = torch.full_like(y, float("nan"))
        form.Mult(dev(x), y2)
        assert torch.equal(y, y2)
        if bz == 1:
            d = torch.empty_like(y)
            form.AssembleDiagonal(d)
            assert relerr(host(d), op.diagonal()) < 1e-13
            assert relerr(form.qdata(E.DIFFUSION), op.D) < 1e-13
            assert relerr(form.qdata(E.MASS)[:, 0, :], op.M) < 1e-13


@pytest.mark.parametrize("mesh_name", ["nonaligned", "fichera_r1", "cart_bricks", "cart_130", "trilinear"])
@pytest.mark.parametrize("order", [1, 2, 3, 4])
@pytest.mark.parametrize("compress", [True, False])
def test_affine_geometry_layout(mesh_name, order, compress):
    """AFFINE qdata (constant element geometry + one (W beta, W alpha detJ) pair per point) is
    chosen exactly for parallelepiped meshes with both integrators -- blocked for the p <= 2
    thread-per-element kernel, element-ordered (AFFINE_E) for the p >= 3 line / brick
    kernels -- and the operator, its diagonal and the reference-layout qdata match the
    oracle either way; non-affine (trilinear) elements get the TRILINEAR layout (map coefficients
    per element, J evaluated per point; TRILINEAR_E at p >= 3); compression off keeps the full
    per-point layout."""
    m = make_mesh(mesh_name)
    fes, form, op = build_pair(m, order, "bio_a", "fn", compress_geometry=compress)
    affine = mesh_name != "trilinear" and AFFINE_ON
    nq = (order + 2) ** 3
    if order <= 2:
        want = E.QLAYOUT_AFFINE if (affine and compress) else E.QLAYOUT_BLOCKED
        if mesh_name == "trilinear" and compress:
            want = E.QLAYOUT_TRILINEAR
    else:
        want = E.QLAYOUT_AFFINE_E if (affine and compress) else E.QLAYOUT_NATIVE
        if mesh_name == "trilinear" and compress:
            want = E.QLAYOUT_TRILINEAR_E
    assert form.info()["layout"] == want
    if want == E.QLAYOUT_AFFINE:
        assert form.qdata_bytes() == 8 * 64 * ((fes.ne + 63) // 64) * (6 + 2 * nq)
    elif want == E.QLAYOUT_AFFINE_E:
        assert form.qdata_bytes() == 8 * fes.ne * (6 + 2 * nq)
    elif want == E.QLAYOUT_TRILINEAR:
        assert form.qdata_bytes() == 8 * 64 * ((fes.ne + 63) // 64) * (22 + 2 * nq)
    elif want == E.QLAYOUT_TRILINEAR_E:
        assert form.qdata_bytes() == 8 * fes.ne * (21 + 2 * nq)
    x = np.random.default_rng(41).uniform(-1, 1, fes.ndofs)
    y = torch.full((fes.ndofs,), float("nan"), dtype=torch.float64, device="cuda")
    form.Mult(dev(x), y)
    assert relerr(host(y), op.mult(x)) <= RTOL
    d = torch.empty(fes.ndofs, dtype=torch.float64, device="cuda")
    form.AssembleDiagonal(d)
    assert relerr(host(d), op.diagonal()) < 1e-13
    assert relerr(form.qdata(E.DIFFUSION), op.D) < 1e-13
    assert relerr(form.qdata(E.MASS)[:, 0, :], op.M) < 1e-13


def test_single_integrator_layouts():
    """A mass-only form keeps the BLOCKED mass stream (already 8 B per point, W alpha det J); a
    diffusion-only form (ex16's K) gets the compressed AFFINE layout with 8-byte points."""
    m = make_mesh("nonaligned")
    for a, b, want in ((2.5, None, E.QLAYOUT_BLOCKED), (None, 0.7, E.QLAYOUT_AFFINE)):
        fes, form, op = build_pair(m, 2, a, b, kernel=E.KERNEL_TPE)
        assert form.info()["layout"] == want
        x = np.random.default_rng(2).uniform(-1, 1, fes.ndofs)
        y = torch.empty(fes.ndofs, dtype=torch.float64, device="cuda")
        form.Mult(dev(x), y)
        assert relerr(host(y), op.mult(x)) <= RTOL


def test_affine_wpe_reads_compressed_layout():
    """The workgroup-per-element pieces (E-vector AddMultPA) read AFFINE qdata through the
    layout-generic accessors: same per-integrator results as the oracle."""
    m = make_mesh("cart_130")
    fes, form, op = build_pair(m, 2, "bio_a", "fn", kernel=E.KERNEL_TPE)
    assert form.info()["layout"] == (E.QLAYOUT_AFFINE if AFFINE_ON else E.QLAYOUT_BLOCKED)
    nd = fes.nd
    xe = np.random.default_rng(3).uniform(-1, 1, (fes.ne, nd))
    for kind, ref in ((E.MASS, O.mass_apply(op.B, op.M, xe)), (E.DIFFUSION, O.diffusion_apply(op.B, op.G, op.D, xe))):
        ye = torch.zeros(fes.ne * nd, dtype=torch.float64, device="cuda")
        form.IntegratorAddMultPA(kind, dev(xe), ye)
        assert relerr(host(ye).reshape(fes.ne, nd), ref) <= RTOL


@pytest.mark.parametrize("order", [1, 2])
def test_cross_wave_face_assembly(order):
    """AFFINE thread-per-element kernels also assemble the faces shared by the 4 bricks of a
    workgroup through LDS: fewer shared dofs / partial slots than the per-wave plan of the
    full layout on the same mesh, and the same operator and diagonal."""
    m = E.Mesh.MakeCartesian3D(16, 16, 8)      # 32 complete 4x4x4 bricks, 8 workgroups
    fa, form_a, op = build_pair(m, order, "bio_a", "fn", kernel=E.KERNEL_TPE)
    fb, form_b, _ = build_pair(m, order, "bio_a", "fn", kernel=E.KERNEL_TPE, compress_geometry=False)
    if XWAVE_ON:
        assert form_a.info()["layout"] == E.QLAYOUT_AFFINE and form_b.info()["layout"] == E.QLAYOUT_BLOCKED
        (sh_a, sl_a), (sh_b, sl_b) = form_a.ScatterInfo(), form_b.ScatterInfo()
        assert sh_a < sh_b and sl_a < sl_b
    x = np.random.default_rng(9).uniform(-1, 1, fa.ndofs)
    for form in (form_a, form_b):
        y = torch.full((fa.ndofs,), float("nan"), dtype=torch.float64, device="cuda")
        form.Mult(dev(x), y)
        assert relerr(host(y), op.mult(x)) <= RTOL
        d = torch.empty(fa.ndofs, dtype=torch.float64, device="cuda")
        form.AssembleDiagonal(d)
        assert relerr(host(d), op.diagonal()) < 1e-13


@pytest.mark.parametrize("mesh_name", ["fichera_r1", "cart_bricks", "trilinear"])
@pytest.mark.parametrize("order", [1, 2, 3, 4])
@pytest.mark.parametrize("compress", [True, False])
def test_attribute_markers(mesh_name, order, compress):
    """"PA Markers" (test_pa_kernels.cpp:696-750): attributes 1 + i % 2, the MassIntegrator
    restricted to attribute 2 by the marker {0, 1} (and, second form, the DiffusionIntegrator
    to attribute 1), through the C ABI's marked integrators, against the oracle's masked
    MultInternal (AddMultWithMarkers, bilinearform_ext.cpp:753-774,807-847) and the
    diagonal of the masked operator; AFFINE and full-layout qdata, fused TPE / line kernels."""
    m = make_mesh(mesh_name)
    m.SetAttributes(1 + np.arange(m.GetNE()) % 2)
    attr = m.GetAttributes()
    fes = E.H1Space(m, order)
    en = m.element_nodes()
    q1d = O.default_q1d(order)
    c = coeff_function(O.quad_points(en, q1d))
    op = O.OracleOperator(en, fes.gather_map(), fes.ndofs, order, alpha=c, beta=c)
    x = np.random.default_rng(3).uniform(-1, 1, fes.ndofs)
    # (mass marker, diffusion marker, diffusion added first)
    for mm, dm, dfirst in (([0, 1], None, False), (None, [1, 0], False), ([0, 1], None, True)):
        form = E.BilinearForm(fes, compress_geometry=compress)
        mi = E.MassIntegrator(E.QuadratureCoefficient(dev(c.reshape(fes.ne, -1))))
        di = E.DiffusionIntegrator(E.QuadratureCoefficient(dev(c.reshape(fes.ne, -1))))
        seq = [(di, dm, "diffusion"), (mi, mm, "mass")] if dfirst else [(mi, mm, "mass"), (di, dm, "diffusion")]
        for integ, mk, _ in seq:
            form.AddDomainIntegrator(integ, mk)
        form.Assemble()
        y = torch.empty(fes.ndofs, dtype=torch.float64, device="cuda")
        form.Mult(dev(x), y)
        ref = op.mult_markers(x, attr, mass_marker=mm, diff_marker=dm)
        assert relerr(host(y), ref) <= RTOL
        # the reference's diagonal (bilinearform_ext.cpp:370-411): a marked integrator zeroes its excluded
        # elements of the shared localY, earlier integrators' contributions included
        d = torch.empty_like(y)
        form.AssembleDiagonal(d)
        dh = host(d)
        assert relerr(dh, op.diagonal_markers(attr, [(k, mk) for _, mk, k in seq])) < 1e-13
        if seq[1][1] is None:  # no later marker: the masked operator's own diagonal, e_i^T A e_i
            for i in np.random.default_rng(4).choice(fes.ndofs, 5, replace=False):
                e = np.zeros(fes.ndofs)
                e[i] = 1.0
                assert abs(dh[i] - op.mult_markers(e, attr, mass_marker=mm, diff_marker=dm)[i]) <= 1e-12 * np.abs(dh).max()
        # Mult after the diagonal: the form's own qdata is back
        form.Mult(dev(x), y)
        assert relerr(host(y), ref) <= RTOL


def test_attribute_marker_errors():
    """A marked integrator needs the attributes, and every attribute must be within the marker
    (the reference verifies marker sizes against attributes.Max())."""
    m = make_mesh("nonaligned")
    fes = E.H1Space(m, 2)
    form = E.BilinearForm(fes)
    form.AddDomainIntegrator(E.MassIntegrator(), [1])
    m.SetAttributes(np.full(m.GetNE(), 2))
    with pytest.raises(E.ECM2Error):
        form.Assemble()


def test_rejected_duplicate_integrator_keeps_marker():
    """A second MassIntegrator / DiffusionIntegrator is rejected (ERR_UNSUPPORTED) and leaves the
    installed integrator, its coefficient and its attribute marker unchanged."""
    m = make_mesh("cart_bricks")
    m.SetAttributes(1 + np.arange(m.GetNE()) % 2)
    fes = E.H1Space(m, 2)
    en = m.element_nodes()
    P = O.quad_points(en, O.default_q1d(2))
    a, c = alpha_bioheat(P), coeff_function(P)
    form = E.BilinearForm(fes)
    form.AddDomainIntegrator(E.MassIntegrator(E.QuadratureCoefficient(dev(a.reshape(fes.ne, -1)))))
    form.AddDomainIntegrator(E.DiffusionIntegrator(E.QuadratureCoefficient(dev(c.reshape(fes.ne, -1)))), [1, 0])
    with pytest.raises(E.ECM2Error):
        form.AddDomainIntegrator(E.DiffusionIntegrator(E.ConstantCoefficient(9.0)))  # unmarked, other coefficient
    with pytest.raises(E.ECM2Error):
        form.AddDomainIntegrator(E.MassIntegrator(E.ConstantCoefficient(9.0)), [0, 1])
    form.Assemble()
    x = np.random.default_rng(3).uniform(-1, 1, fes.ndofs)
    y = torch.empty(fes.ndofs, dtype=torch.float64, device="cuda")
    form.Mult(dev(x), y)
    op = O.OracleOperator(en, fes.gather_map(), fes.ndofs, 2, alpha=a, beta=c)
    assert relerr(host(y), op.mult_markers(x, m.GetAttributes(), diff_marker=[1, 0])) <= RTOL


@pytest.mark.parametrize("order", [1, 2])
@pytest.mark.parametrize("mesh_name", ["trilinear", "trilinear_big"])
@pytest.mark.parametrize("numbering", [E.NUMBERING_STRUCTURED, E.NUMBERING_ENTITY])
def test_trilinear_layout_on_the_fly_geometry(order, mesh_name, numbering):
    """TRILINEAR layout (general trilinear hexes, p <= 2): the fused kernel evaluates J, adj(J)
    and det J at every point from the element's map coefficients -- the operator, the diagonal,
    the E-vector integrator applies and the reference-layout qdata all match the oracle's
    setup + apply (bilininteg_diffusion_kernels.cpp:243-367, bilininteg_mass_pa.cpp:62-78),
    on lattice-addressed and map-addressed blocks, and with an attribute marker."""
    if mesh_name == "trilinear":
        m = make_mesh("trilinear")
    else:
        m = E.Mesh.MakeCartesian3D(8, 8, 9, 1.0, 1.0, 9 / 8)  # complete 4x4x4 bricks + a ragged layer
        V = m.vertices()
        inner = np.all((V > 1e-9) & (V < np.array([1.0, 1.0, 9 / 8]) - 1e-9), axis=1)
        V[inner] += 0.03 * np.random.default_rng(8).uniform(-1, 1, (int(inner.sum()), 3))
        m.set_vertices(V)
    fes, form, op = build_pair(m, order, "bio_a", "fn", numbering=numbering)
    assert form.info()["layout"] == E.QLAYOUT_TRILINEAR
    x = np.random.default_rng(5).uniform(-1, 1, fes.ndofs)
    y = torch.full((fes.ndofs,), float("nan"), dtype=torch.float64, device="cuda")
    form.Mult(dev(x), y)
    assert relerr(host(y), op.mult(x)) <= RTOL
    d = torch.empty_like(y)
    form.AssembleDiagonal(d)
    assert relerr(host(d), op.diagonal()) < 1e-13
    assert relerr(form.qdata(E.DIFFUSION), op.D) < 1e-13
    assert relerr(form.qdata(E.MASS)[:, 0, :], op.M) < 1e-13
    xe = np.random.default_rng(6).uniform(-1, 1, (fes.ne, fes.nd))
    ye = torch.zeros(fes.ne * fes.nd, dtype=torch.float64, device="cuda")
    form.IntegratorAddMultPA(E.DIFFUSION, dev(xe), ye)
    assert relerr(host(ye).reshape(fes.ne, fes.nd), O.diffusion_apply(op.B, op.G, op.D, xe)) <= RTOL
    if mesh_name == "trilinear_big":
        lat, units, _ = form.AddressingInfo()
        if numbering == E.NUMBERING_STRUCTURED:
            assert lat > 0  # lattice-addressed blocks run the TRILINEAR kernel too
        m.SetAttributes(1 + np.arange(m.GetNE()) % 2)
        f2 = E.BilinearForm(fes)
        en = m.element_nodes()
        P = O.quad_points(en, O.default_q1d(order))
        a, c = alpha_bioheat(P), coeff_function(P)
        f2.AddDomainIntegrator(E.MassIntegrator(E.QuadratureCoefficient(dev(a.reshape(fes.ne, -1)))), [0, 1])
        f2.AddDomainIntegrator(E.DiffusionIntegrator(E.QuadratureCoefficient(dev(c.reshape(fes.ne, -1)))))
        f2.Assemble()
        assert f2.info()["layout"] == E.QLAYOUT_TRILINEAR
        f2.Mult(dev(x), y)
        opm = O.OracleOperator(en, fes.gather_map(), fes.ndofs, order, alpha=a, beta=c)
        assert relerr(host(y), opm.mult_markers(x, m.GetAttributes(), mass_marker=[0, 1])) <= RTOL


def test_jacobians_not_trilinear_keep_per_point_layout():
    """Jacobians that no trilinear map produces (one point of one element perturbed, as on a
    curved mesh) fail the fit's per-point check: the form keeps the full per-point layout."""
    m = make_mesh("trilinear")
    fes = E.H1Space(m, 2)
    _, J, _ = O.geom(m.element_nodes(), O.default_q1d(2))
    J = np.array(J)
    J[7, 0, 1, 5] *= 1.0 + 1e-6
    form = E.BilinearForm(fes, geometry="jacobians")
    form.SetJacobians(dev(J))
    form.AddDomainIntegrator(E.MassIntegrator(E.ConstantCoefficient(3.0)))
    form.AddDomainIntegrator(E.DiffusionIntegrator(E.ConstantCoefficient(0.5)))
    form.Assemble()
    assert form.info()["layout"] == E.QLAYOUT_BLOCKED
