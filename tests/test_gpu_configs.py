"""GPU parity on the BASELINE configurations as the build runs them by default.

* configs[2] (C3): fichera.mesh refined 6x as the bench runs it (14.9M DoF, the Pennes k(T)
  re-assembly), and refined 2x / 3x (448 / 3,584 elements) at p = 1, 2 with the
  default element order, so the face-linked 4x4x4 bricks derived from the gather map and the
  cross-wave LDS face merge run on a non-lattice mesh; Mult and diagonal against the oracle;
  the Pennes k(T) grid-function coefficient and Jacobi-PCG together on r3 against the
  oracle's PCG (the reference pins PA == FA on fichera: test_pa_kernels.cpp:641-694).
* Known answers on the reference's own fichera fixture through the HIP path: 1^T M 1 = |fichera|
  = 7 and x^T K x = 7 |g|^2 for the linear x = g . X (H1 interpolates it exactly).
* configs[4] (C5): p = 4 Cartesian 32^3 (2.15M DoF) and 68^3 (20.3M DoF, the bench size), all
  elements in 2 x 2 x 1 bricks, against the oracle; the SDIRK33 step (ode.cpp:834-859) at p = 4
  against the oracle's stepping.
* configs[3] (C4): the 8-way z-slab split of a 16^3 p = 2 mesh (loopback group, both
  decompositions) against the serial oracle, and of the full 108^3 mesh (10.2M DoF) as the 8-GPU
  bench runs it, each member's rows alone and the whole group.
* Lattice addressing (the fused kernels compute dofs from 5 ints per block / brick on a
  lattice-numbered mesh) against the map-reading path on the same mesh with the entity
  numbering, p = 1, 2 and 4, Mult and diagonal.
* The boundary's MultTranspose (bilinearform_ext.hpp:99) and AddMult; the device Pennes
  perfusion law (parity-unpinned law, pinned projection); the distributed form's graph cache
  across re-assembly.
Bar: ||y - y_ref||_inf / ||y_ref||_inf <= RTOL = 1e-12 (FP64)."""
import numpy as np
import pytest

import ecm2_amd as E
import oracle as O
import bioheat as BH
import ode as ODE
from helpers import GOLDEN, RTOL, alpha_bioheat, coeff_function, k_of_T, nonaligned, relerr, temperature

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


def fichera(refinements):
    m = E.Mesh(f"{GOLDEN}/fichera.mesh")
    for _ in range(refinements):
        m.UniformRefinement()
    return m


def quad_coeff(fes, values):
    return E.QuadratureCoefficient(dev(np.asarray(values).reshape(fes.ne, -1)))


# ---------------------------------------------------------------------------------------
# configs[2]: fichera refined, default path (face-linked bricks + cross-wave merge)
# ---------------------------------------------------------------------------------------
@pytest.mark.parametrize("refine", [2, 3])
@pytest.mark.parametrize("order", [1, 2])
def test_c3_fichera_default_path(refine, order):
    m = fichera(refine)
    assert m.GetNE() == 7 * 8 ** refine
    fes = E.H1Space(m, order)
    # every element of a refined fichera lies in a face-linked 4x4x4 brick
    perm = fes.element_order_faces()
    assert sorted(perm.tolist()) == list(range(fes.ne))
    en = m.element_nodes()
    q1d = O.default_q1d(order)
    P = O.quad_points(en, q1d)
    a, b = alpha_bioheat(P), k_of_T(temperature(P))
    form = E.BilinearForm(fes)                       # defaults: auto kernel, auto element order
    form.AddDomainIntegrator(E.MassIntegrator(quad_coeff(fes, a)))
    form.AddDomainIntegrator(E.DiffusionIntegrator(quad_coeff(fes, b)))
    form.Assemble()
    info = form.info()
    assert info["kernel"] == E.KERNEL_TPE and info["layout"] == E.QLAYOUT_AFFINE
    native = E.BilinearForm(fes, element_order="native")
    native.AddDomainIntegrator(E.MassIntegrator(quad_coeff(fes, a)))
    native.AddDomainIntegrator(E.DiffusionIntegrator(quad_coeff(fes, b)))
    native.Assemble()
    # the brick order assembles faces in-wave and across waves: far fewer shared dofs
    assert form.ScatterInfo()[0] < native.ScatterInfo()[0] // 2
    op = O.OracleOperator(en, fes.gather_map(), fes.ndofs, order, alpha=a, beta=b)
    x = np.random.default_rng(refine * 10 + order).uniform(-1, 1, fes.ndofs)
    for f in (form, native):
        y = torch.full((fes.ndofs,), float("nan"), dtype=torch.float64, device="cuda")
        f.Mult(dev(x), y)
        assert relerr(host(y), op.mult(x)) <= RTOL
        d = torch.full_like(y, float("nan"))
        f.AssembleDiagonal(d)
        assert relerr(host(d), op.diagonal()) < 1e-13


@pytest.mark.parametrize("jacobi", [True, False])
def test_c3_fichera_pennes_pcg(jacobi):
    """k(T) from an H1 temperature field (GridFunctionCoefficient projection + the Pennes law,
    re-assembled on the device) inside the constrained Jacobi-PCG, r3 = 3,584 elements."""
    m = fichera(3)
    order = 2
    fes = E.H1Space(m, order)
    en = m.element_nodes()
    q1d = O.default_q1d(order)
    T = temperature(fes.dof_coords())
    scale, slope, tref = 0.5 * 0.05, 0.0012, 37.0
    form = E.BilinearForm(fes)
    form.AddDomainIntegrator(E.MassIntegrator(E.ConstantCoefficient(1.0)))
    form.AddDomainIntegrator(E.DiffusionIntegrator(E.AffineGridFunctionCoefficient(dev(T), scale, slope, tref)))
    form.Assemble()
    beta = BH.affine_law(BH.temperature_at_quadrature(T, fes.gather_map(), order, q1d), scale, slope, tref)
    op = O.OracleOperator(en, fes.gather_map(), fes.ndofs, order, alpha=1.0, beta=beta)
    ess = fes.boundary_dofs()
    b = np.random.default_rng(4).uniform(-1, 1, fes.ndofs)
    x = torch.empty(fes.ndofs, dtype=torch.float64, device="cuda")
    it, _ = form.PCG(dev(b), x, ess=dev(ess, torch.int32), rel_tol=1e-12, max_iter=3000, jacobi=jacobi)
    xr, itr, _ = op.pcg(b, ess, rel_tol=1e-12, max_iter=3000, jacobi=jacobi)
    # rounding differences move the iteration at which the 1e-12 test is first met by a few
    assert abs(it - itr) <= max(2, 0.05 * itr)
    assert relerr(host(x), xr) < 1e-9


def test_c3_full_size():
    """configs[2] at the bench size: fichera.mesh refined 6x (1.84M elements, 14.9M DoF), p = 2,
    default path (face-linked bricks, cross-wave merge), heat capacity as a quadrature coefficient
    and k(T) from an H1 temperature field re-assembled on the device, against the oracle: the
    Mult, and 8 iterations of the constrained Jacobi-PCG the bench times."""
    m = fichera(6)
    order, q1d = 2, O.default_q1d(2)
    fes = E.H1Space(m, order)
    assert fes.ndofs == 14877441
    en = m.element_nodes()
    P = O.quad_points(en, q1d)
    a = alpha_bioheat(P)
    del P
    T = temperature(fes.dof_coords())
    scale, slope, tref = 0.5 * 0.05, 0.0012, 37.0
    form = E.BilinearForm(fes)
    form.AddDomainIntegrator(E.MassIntegrator(quad_coeff(fes, a)))
    form.AddDomainIntegrator(E.DiffusionIntegrator(E.AffineGridFunctionCoefficient(dev(T), scale, slope, tref)))
    form.Assemble()
    assert form.info()["kernel"] == E.KERNEL_TPE and form.info()["layout"] == E.QLAYOUT_AFFINE
    x = np.random.default_rng(6).uniform(-1, 1, fes.ndofs)
    y = torch.full((fes.ndofs,), float("nan"), dtype=torch.float64, device="cuda")
    form.Mult(dev(x), y)
    yh = host(y)
    del y
    beta = BH.affine_law(BH.temperature_at_quadrature(T, fes.gather_map(), order, q1d), scale, slope, tref)
    op = O.OracleOperator(en, fes.gather_map(), fes.ndofs, order, alpha=a, beta=beta)
    assert relerr(yh, op.mult(x)) <= RTOL
    # the bench's C3 solve at full size: constrained Jacobi-PCG, a fixed 8 iterations (rel_tol 0)
    # on both sides (CGSolver::Mult, solvers.cpp:869-1004, with ConstrainedOperator DIAG_ONE)
    ess = fes.boundary_dofs()
    b = np.random.default_rng(2).uniform(-1, 1, fes.ndofs)
    xs = torch.empty(fes.ndofs, dtype=torch.float64, device="cuda")
    it, _ = form.PCG(dev(b), xs, ess=dev(ess, torch.int32), rel_tol=0.0, max_iter=8, jacobi=True)
    xr, itr, _ = op.pcg(b, ess, rel_tol=0.0, max_iter=8, jacobi=True)
    assert it == itr == 8
    assert relerr(host(xs), xr) < 1e-10


@pytest.mark.parametrize("refine", [1, 2, 3])
@pytest.mark.parametrize("order", [1, 2, 3])
def test_fichera_known_answers(refine, order):
    """On the reference's data/fichera.mesh (7 unit cubes): 1^T M 1 = 7 and, for x = g . X
    (linear: exactly in every H1 space), x^T K x = |g|^2 7 and K x = 0 in the interior dofs'
    sense of sum(K x) = 0 (K 1 = 0)."""
    m = fichera(refine)
    fes = E.H1Space(m, order)
    X = fes.dof_coords()
    M = E.BilinearForm(fes)
    M.AddDomainIntegrator(E.MassIntegrator(E.ConstantCoefficient(1.0)))
    M.Assemble()
    K = E.BilinearForm(fes)
    K.AddDomainIntegrator(E.DiffusionIntegrator(E.ConstantCoefficient(1.0)))
    K.Assemble()
    one = torch.ones(fes.ndofs, dtype=torch.float64, device="cuda")
    y = torch.empty_like(one)
    M.Mult(one, y)
    assert abs(float(y.sum()) - 7.0) < 1e-12 * 7.0
    g = np.array([0.3, -1.1, 0.7])
    x = dev(X @ g)
    K.Mult(x, y)
    assert abs(float(torch.dot(x, y)) - 7.0 * g @ g) < 1e-11 * 7.0 * (g @ g)
    K.Mult(one, y)
    assert float(y.abs().max()) < 1e-12


# ---------------------------------------------------------------------------------------
# configs[4]: p = 4 at size, and the SDIRK step at p = 4
# ---------------------------------------------------------------------------------------
def test_c5_p4_cartesian_32():
    n = 32
    m = E.Mesh.MakeCartesian3D(n, n, n)
    fes = E.H1Space(m, 4, E.NUMBERING_STRUCTURED)
    assert fes.ndofs == (4 * n + 1) ** 3
    en = m.element_nodes()
    P = O.quad_points(en, 6)
    a, b = alpha_bioheat(P), k_of_T(temperature(P))
    form = E.BilinearForm(fes)
    form.AddDomainIntegrator(E.MassIntegrator(quad_coeff(fes, a)))
    form.AddDomainIntegrator(E.DiffusionIntegrator(quad_coeff(fes, b)))
    form.Assemble()
    assert form.info()["kernel"] == E.KERNEL_LINE and form.info()["layout"] == E.QLAYOUT_AFFINE_E
    assert form.BrickInfo() == (fes.ne // 4, 1)      # every element in a 2 x 2 x 1 brick
    lat, units, _ = form.AddressingInfo()
    assert lat == units == fes.ne // 4                 # every brick lattice-addressed (no map reads)
    x = np.random.default_rng(32).uniform(-1, 1, fes.ndofs)
    y = torch.full((fes.ndofs,), float("nan"), dtype=torch.float64, device="cuda")
    form.Mult(dev(x), y)
    op = O.OracleOperator(en, fes.gather_map(), fes.ndofs, 4, alpha=a, beta=b)
    assert relerr(host(y), op.mult(x)) <= RTOL
    y2 = torch.full_like(y, float("nan"))
    form.Mult(dev(x), y2)
    assert torch.equal(y, y2)                         # deterministic scatter


def test_c5_full_size():
    """configs[4] at size: Cartesian 68^3, p = 4 (20.3M DoF), every element in a lattice-addressed
    2 x 2 x 1 brick, against the oracle."""
    n = 68
    m = E.Mesh.MakeCartesian3D(n, n, n)
    fes = E.H1Space(m, 4, E.NUMBERING_STRUCTURED)
    assert fes.ndofs == 20346417
    en = m.element_nodes()
    P = O.quad_points(en, 6)
    a, b = alpha_bioheat(P), k_of_T(temperature(P))
    del P
    form = E.BilinearForm(fes)
    form.AddDomainIntegrator(E.MassIntegrator(quad_coeff(fes, a)))
    form.AddDomainIntegrator(E.DiffusionIntegrator(quad_coeff(fes, b)))
    form.Assemble()
    assert form.BrickInfo() == (fes.ne // 4, 1) and form.AddressingInfo()[0] == fes.ne // 4
    x = np.random.default_rng(68).uniform(-1, 1, fes.ndofs)
    y = torch.full((fes.ndofs,), float("nan"), dtype=torch.float64, device="cuda")
    form.Mult(dev(x), y)
    yh = host(y)
    del form, y
    op = O.OracleOperator(en, fes.gather_map(), fes.ndofs, 4, alpha=a, beta=b)
    assert relerr(yh, op.mult(x)) <= RTOL


def test_c5_full_size_drop_in():
    """configs[4] size in the drop-in configuration at p = 4: MakeCartesian3D's space-filling-curve
    element order and FiniteElementSpace's entity dofs, interior vertices moved (non-affine hexes)
    and the geometry as MFEM Jacobians (set_jacobians, fitted to trilinear maps: TRILINEAR_E, the
    brick kernel evaluating J and adj(J) per point), against the oracle."""
    n = 68
    m = E.Mesh.MakeCartesian3D(n, n, n, sfc_ordering=True)
    V = m.vertices()
    h = 1.0 / n
    inner = np.all((V > 0.5 * h) & (V < 1.0 - 0.5 * h), axis=1)
    V[inner] += 0.15 * h * np.random.default_rng(11).uniform(-1, 1, (int(inner.sum()), 3))
    m.set_vertices(V)
    fes = E.H1Space(m, 4, E.NUMBERING_ENTITY)
    assert fes.ndofs == 20346417
    en = m.element_nodes()
    P = O.quad_points(en, 6)
    a, b = alpha_bioheat(P), k_of_T(temperature(P))
    del P
    form = E.BilinearForm(fes, geometry="jacobians")
    form.SetJacobians(m.jacobians(6))
    form.AddDomainIntegrator(E.MassIntegrator(quad_coeff(fes, a)))
    form.AddDomainIntegrator(E.DiffusionIntegrator(quad_coeff(fes, b)))
    form.Assemble()
    assert form.info()["layout"] == E.QLAYOUT_TRILINEAR_E and form.BrickInfo()[0] > 0
    x = np.random.default_rng(69).uniform(-1, 1, fes.ndofs)
    y = torch.full((fes.ndofs,), float("nan"), dtype=torch.float64, device="cuda")
    form.Mult(dev(x), y)
    yh = host(y)
    del form, y
    op = O.OracleOperator(en, fes.gather_map(), fes.ndofs, 4, alpha=a, beta=b)
    assert relerr(yh, op.mult(x)) <= RTOL


SMOOTH_TOL = 1e-12  # converged stages (rel_tol 1e-12): measured 5.8e-15 (profiles/r6/gpu17_tests.txt)


def _serial_form(fes, P, alpha, beta):
    f = E.BilinearForm(fes)
    if alpha is not None:
        f.AddDomainIntegrator(E.MassIntegrator(quad_coeff(fes, alpha)))
    if beta is not None:
        f.AddDomainIntegrator(E.DiffusionIntegrator(quad_coeff(fes, beta)))
    f.Assemble()
    return f


@pytest.mark.parametrize("ode_type", [23, 21])
def test_c5_sdirk_step_p4(ode_type):
    """Two SDIRK33 (and backward Euler) steps of M du/dt = -K u at p = 4 with Dirichlet dofs
    held, device ode_step (bricks + line kernel on a non-aligned mesh) against the oracle's
    stepping with the oracle's PCG stage solves (ode.cpp:682-686, 834-859; ex16p.cpp:373-470)."""
    m = E.Mesh.MakeCartesian3D(6, 4, 5)
    m.set_vertices(nonaligned(m.vertices()))
    order, dt = 4, 0.02
    fes = E.H1Space(m, order)
    en = m.element_nodes()
    P = O.quad_points(en, O.default_q1d(order))
    alpha = 2.0 + np.sin(P[..., 0]) * np.cos(P[..., 1])
    beta = coeff_function(P)
    c = E.ode_implicit_coeff(ode_type)
    T = _serial_form(fes, P, alpha, c * dt * beta)
    K = _serial_form(fes, P, None, beta)
    assert T.BrickInfo()[0] > 0
    Tr = O.OracleOperator(en, fes.gather_map(), fes.ndofs, order, alpha=alpha, beta=c * dt * beta)
    Kr = O.OracleOperator(en, fes.gather_map(), fes.ndofs, order, beta=beta)
    ess = fes.boundary_dofs()
    X = fes.dof_coords()
    u0 = 37.0 + 20.0 * np.exp(-4.0 * np.sum((X - 0.5) ** 2, axis=1))

    def solve(us):
        rhs = -Kr.mult(us)
        rhs[ess] = 0.0
        return Tr.pcg(rhs, ess, rel_tol=1e-13, max_iter=20000)[0]

    ur = u0.copy()
    for _ in range(2):
        ur = ODE.step(ode_type, solve, ur, dt)
    u = dev(u0)
    essd = dev(ess, torch.int32)
    for _ in range(2):
        ns, it, conv = E.ode_step(ode_type, E.Operator(T), E.Operator(K), dt, u, ess=essd, rel_tol=1e-13,
                                  max_iter=20000)
        assert conv and ns == {21: 1, 23: 3}[ode_type]
    uh = host(u)
    assert np.array_equal(uh[ess], u0[ess])
    assert relerr(uh - u0, ur - u0) < 1e-9


def test_c5_sdirk_step_full_size():
    """configs[4]'s implicit time step at size: one SDIRK33 step (ode.cpp:834-859, ex16p.cpp:373-470)
    of M du/dt = -K u on Cartesian 68^3 at p = 4 (20.3M DoF, every element in a lattice-addressed
    2 x 2 x 1 brick), T = M_alpha + c dt K_beta and K = K_beta as the bench's forms, Dirichlet dofs
    held; each of the three stage solves a constrained Jacobi-PCG with a fixed 8 iterations (rel_tol
    0) on both sides -- the device ode_step against oracle/ode.py's SDIRK33 over the oracle's PCG."""
    n, order, dt, iters = 68, 4, 0.02, 8
    m = E.Mesh.MakeCartesian3D(n, n, n)
    fes = E.H1Space(m, order, E.NUMBERING_STRUCTURED)
    assert fes.ndofs == 20346417
    en = m.element_nodes()
    P = O.quad_points(en, O.default_q1d(order))
    alpha, beta = alpha_bioheat(P) / 3.6e6, k_of_T(temperature(P))
    del P
    c = E.ode_implicit_coeff(23)
    T = _serial_form(fes, None, alpha, c * dt * beta)
    K = _serial_form(fes, None, None, beta)
    assert T.BrickInfo() == (fes.ne // 4, 1) and T.info()["layout"] == E.QLAYOUT_AFFINE_E
    ess = fes.boundary_dofs()
    # a rough state (uniform random): K u0 without cancellation, so the comparison measures the step's
    # algebra rather than the rounding of a near-zero Laplacian amplified by 24 unconverged CG iterations
    u0 = np.random.default_rng(68).uniform(-1.0, 1.0, fes.ndofs)
    u = dev(u0)
    ns, it, conv = E.ode_step(23, E.Operator(T), E.Operator(K), dt, u, ess=dev(ess, torch.int32), rel_tol=0.0,
                              max_iter=iters)
    assert ns == 3 and it == 3 * iters and not conv   # fixed iteration count: "not converged" by design
    uh = host(u)
    del T, K, u
    Tr = O.OracleOperator(en, fes.gather_map(), fes.ndofs, order, alpha=alpha, beta=c * dt * beta)
    Kr = O.OracleOperator(en, fes.gather_map(), fes.ndofs, order, beta=beta)
    del alpha, beta

    def solve(us):
        rhs = -Kr.mult(us)
        rhs[ess] = 0.0
        xs, itr, _ = Tr.pcg(rhs, ess, rel_tol=0.0, max_iter=iters)
        assert itr == iters
        return xs

    ur = ODE.step(23, solve, u0, dt)
    assert np.array_equal(uh[ess], u0[ess])
    assert relerr(uh - u0, ur - u0) < 1e-9


def _c5_smooth_step(g, rel_tol, max_iter, shift=0.0):
    """One SDIRK33 step at 68^3 p = 4 from u0 = 37 + 20 exp(-4 |x - 1/2|^2) - shift through the device forms;
    returns (relerr of u1 - u0 at the fixture's dofs against its oracle values, the device's stage iterations,
    converged)."""
    n, order, dt = 68, 4, 0.02
    m = E.Mesh.MakeCartesian3D(n, n, n)
    fes = E.H1Space(m, order, E.NUMBERING_STRUCTURED)
    assert fes.ndofs == int(g["ndofs"])
    en = m.element_nodes()
    P = O.quad_points(en, O.default_q1d(order))
    alpha, beta = alpha_bioheat(P) / 3.6e6, k_of_T(temperature(P))
    del P
    c = E.ode_implicit_coeff(23)
    T = _serial_form(fes, None, alpha, c * dt * beta)
    K = _serial_form(fes, None, None, beta)
    del alpha, beta
    ess = fes.boundary_dofs()
    X = fes.dof_coords()
    u0 = 37.0 + 20.0 * np.exp(-4.0 * np.sum((X - 0.5) ** 2, axis=1)) - shift
    idx = g["idx"]
    assert np.array_equal(u0[idx], g["u0"])
    u = dev(u0)
    ns, it, conv = E.ode_step(23, E.Operator(T), E.Operator(K), dt, u, ess=dev(ess, torch.int32), rel_tol=rel_tol,
                              max_iter=max_iter)
    assert ns == 3
    uh = host(u)
    assert np.array_equal(uh[ess], u0[ess])
    return relerr(uh[idx] - u0[idx], g["u1"] - g["u0"]), it, conv


def test_c5_sdirk_smooth_converged():
    """configs[4]'s step from the SMOOTH state with converged stage solves: one SDIRK33
    step at 68^3 p = 4 (20.3M DoF) from u0 = 37 + 20 exp(-4 |x - 1/2|^2), each stage a constrained
    Jacobi-PCG to rel_tol 1e-12, against the oracle's step on the same mesh (tests/golden/sdirk_c5_smooth.npz,
    written by profiles/r6/sdirk_smooth_cpu.py --converged: u1 at 20,000 seeded dofs; the oracle needs ~50 min
    on 8 threads).  The oracle against itself with its elements permuted differs by 7.7e-15 here
    (profiles/r6/sdirk_smooth_cpu.txt)."""
    g = np.load(f"{GOLDEN}/sdirk_c5_smooth.npz")
    err, it, conv = _c5_smooth_step(g, 1e-12, 100000)
    print(f"c5 smooth converged SDIRK33: device stage iterations {it} (oracle {g['iterations'].tolist()}), relerr {err:.3e}")
    assert conv
    assert err < SMOOTH_TOL


def test_c5_sdirk_smooth_fixed8():
    """The same smooth-state step with 8 fixed Jacobi-PCG iterations per stage (rel_tol 0), the form of round 5's
    2.9e-7 gap, against the oracle's step (tests/golden/sdirk_c5_smooth_fixed8.npz, written by
    profiles/r6/sdirk_smooth_cpu.py --fixed8-fixture).  The gap is the step's conditioning, not the device:
    (1) the ORACLE's own step from u0 and from u0 - 37 -- the same step in exact arithmetic, K 1 = 0 -- differs by
    3.8e-7 (profiles/r6/sdirk_smooth_cpu_shift.txt) for a change of K u0 of 3.6e-12 relative (the oracle's
    |37 K 1| = 3.3e-13 against |K u0| = 0.092, profiles/r6/sdirk_gap_probe.txt): 8 unconverged iterations amplify
    a relative change of the stage right-hand side ~1e5 times; (2) a smooth state's K u0 cancels ~5 digits
    inside every element, and the device's sum-factorised element products round differently from the oracle's:
    2.4e-12 relative on K u0 (1e5 x that is the 2.3e-7 seen here), 2.5e-15 on a random state; (3) two device
    forms that round alike inside the element (compressed and per-point geometry) agree to 2.3e-10, and with
    converged stage solves device and oracle agree to 5.8e-15 (test_c5_sdirk_smooth_converged).  The bound is
    that self-gap's order, 1e-6."""
    g = np.load(f"{GOLDEN}/sdirk_c5_smooth_fixed8.npz")
    err, it, conv = _c5_smooth_step(g, 0.0, 8)
    print(f"c5 smooth fixed-8 SDIRK33: device iterations {it} (oracle {g['iterations'].tolist()}), relerr {err:.3e}")
    assert it == 24 and not conv
    assert err < 1e-6


# ---------------------------------------------------------------------------------------
# configs[3]: the 8-way split
# ---------------------------------------------------------------------------------------
@pytest.mark.parametrize("decomp", ["rap", "overlap"])
@pytest.mark.parametrize("scatter", ["partials", "atomic"])
def test_c4_eight_way_slabs(decomp, scatter):
    n, nranks, order = 16, 8, 2
    m = E.Mesh.MakeCartesian3D(n, n, n)
    fes = E.H1Space(m, order, E.NUMBERING_STRUCTURED)
    er = E.partition_slabs_z(m, nranks)
    q1d = O.default_q1d(order)
    xg = np.random.default_rng(8).uniform(-1, 1, fes.ndofs)
    forms, parts, xs, ys = [], [], [], []
    for r in range(nranks):
        part = E.Partition(fes, er, r, nranks, decomposition=decomp)
        pf = E.ParBilinearForm(part, scatter=scatter)
        P = E.quadrature_points_subset(m, q1d, part.elems)
        pf.AddDomainIntegrator(E.MassIntegrator(E.QuadratureCoefficient(dev(alpha_bioheat(P).reshape(part.ne_local, -1)))))
        pf.AddDomainIntegrator(E.DiffusionIntegrator(E.QuadratureCoefficient(
            dev(k_of_T(temperature(P)).reshape(part.ne_local, -1)))))
        pf.Assemble()
        forms.append(pf)
        parts.append(part)
        xs.append(dev(xg[part.owned_global]))
        ys.append(torch.full((part.n_owned,), float("nan"), dtype=torch.float64, device="cuda"))
    assert all(p.n_nbrs <= 2 for p in parts) and parts[3].n_nbrs == 2
    group = E.ParGroup(forms)
    for _ in range(2):  # repeated Mults reuse the streams, events and buffers
        group.Mult(xs, ys)
    y = np.full(fes.ndofs, np.nan)
    for part, yt in zip(parts, ys):
        y[part.owned_global] = host(yt)
    Pg = O.quad_points(m.element_nodes(), q1d)
    ref = O.OracleOperator(m.element_nodes(), fes.gather_map(), fes.ndofs, order, alpha=alpha_bioheat(Pg),
                           beta=k_of_T(temperature(Pg))).mult(xg)
    assert relerr(y, ref) <= RTOL


def test_c4_full_size_eight_way_members():
    """configs[3] exactly as the 8-GPU bench runs it: Cartesian 108^3 (10.2M DoF) in 8 z-slabs,
    OVERLAP, the serial schedule; every member's rows alone (ParGroup.MultMember, what one rank
    computes on its GPU) and the whole group against one oracle Mult of the full mesh."""
    n, nranks, order = 108, 8, 2
    m = E.Mesh.MakeCartesian3D(n, n, n)
    fes = E.H1Space(m, order, E.NUMBERING_STRUCTURED)
    assert fes.ndofs == 10218313
    er = E.partition_slabs_z(m, nranks)
    q1d = O.default_q1d(order)
    xg = np.random.default_rng(108).uniform(-1, 1, fes.ndofs)
    forms, parts, xs, ys = [], [], [], []
    for r in range(nranks):
        part = E.Partition(fes, er, r, nranks, decomposition="overlap")
        pf = E.ParBilinearForm(part)
        P = E.quadrature_points_subset(m, q1d, part.elems)
        pf.AddDomainIntegrator(E.MassIntegrator(E.QuadratureCoefficient(dev(alpha_bioheat(P).reshape(part.ne_local, -1)))))
        pf.AddDomainIntegrator(E.DiffusionIntegrator(E.QuadratureCoefficient(
            dev(k_of_T(temperature(P)).reshape(part.ne_local, -1)))))
        pf.Assemble()
        forms.append(pf)
        parts.append(part)
        xs.append(dev(xg[part.owned_global]))
        ys.append(torch.full((part.n_owned,), float("nan"), dtype=torch.float64, device="cuda"))
        del P
    Pg = O.quad_points(m.element_nodes(), q1d)
    ref = O.OracleOperator(m.element_nodes(), fes.gather_map(), fes.ndofs, order, alpha=alpha_bioheat(Pg),
                           beta=k_of_T(temperature(Pg))).mult(xg)
    del Pg
    group = E.ParGroup(forms)
    for r in range(nranks):
        group.MultMember(r, xs, ys)
    y = np.full(fes.ndofs, np.nan)
    for part, yt in zip(parts, ys):
        y[part.owned_global] = host(yt)
    assert relerr(y, ref) <= RTOL
    for yt in ys:
        yt.fill_(float("nan"))
    group.Mult(xs, ys)
    for part, yt in zip(parts, ys):
        y[part.owned_global] = host(yt)
    assert relerr(y, ref) <= RTOL


def _c5_group(m, fes, er, nranks, alpha_fn, beta_fn, q1d):
    """The 8 z-slab members of configs[4] (OVERLAP, the serial schedule), each with its own
    quadrature-point coefficients; alpha_fn / beta_fn map points to values (None: integrator absent)."""
    forms, parts = [], []
    for r in range(nranks):
        part = E.Partition(fes, er, r, nranks, decomposition="overlap")
        pf = E.ParBilinearForm(part)
        P = E.quadrature_points_subset(m, q1d, part.elems)
        if alpha_fn is not None:
            pf.AddDomainIntegrator(E.MassIntegrator(E.QuadratureCoefficient(dev(alpha_fn(P).reshape(part.ne_local, -1)))))
        pf.AddDomainIntegrator(E.DiffusionIntegrator(E.QuadratureCoefficient(dev(beta_fn(P).reshape(part.ne_local, -1)))))
        pf.Assemble()
        forms.append(pf)
        parts.append(part)
        del P
    return forms, parts


def test_c5_full_size_eight_way_members():
    """configs[4] split 8 ways at size: Cartesian 68^3 at p = 4 (20.3M DoF) in 8
    z-slabs (CartesianPartitioning rounding: 8 or 9 element layers per rank), OVERLAP, every rank's
    elements in 2 x 2 x 1 bricks + the line kernel; every member's rows alone (ParGroup.MultMember,
    what one rank computes on its GPU) and the whole group against one oracle Mult of the full mesh
    -- the p = 4 analogue of test_c4_full_size_eight_way_members."""
    n, nranks, order = 68, 8, 4
    m = E.Mesh.MakeCartesian3D(n, n, n)
    fes = E.H1Space(m, order, E.NUMBERING_STRUCTURED)
    assert fes.ndofs == 20346417
    er = E.partition_slabs_z(m, nranks)
    q1d = O.default_q1d(order)
    forms, parts = _c5_group(m, fes, er, nranks, alpha_bioheat, lambda P: k_of_T(temperature(P)), q1d)
    xg = np.random.default_rng(68).uniform(-1, 1, fes.ndofs)
    xs = [dev(xg[p.owned_global]) for p in parts]
    ys = [torch.full((p.n_owned,), float("nan"), dtype=torch.float64, device="cuda") for p in parts]
    Pg = O.quad_points(m.element_nodes(), q1d)
    ref = O.OracleOperator(m.element_nodes(), fes.gather_map(), fes.ndofs, order, alpha=alpha_bioheat(Pg),
                           beta=k_of_T(temperature(Pg))).mult(xg)
    del Pg
    group = E.ParGroup(forms)
    for r in range(nranks):
        group.MultMember(r, xs, ys)
    y = np.full(fes.ndofs, np.nan)
    for part, yt in zip(parts, ys):
        y[part.owned_global] = host(yt)
    assert relerr(y, ref) <= RTOL
    for yt in ys:
        yt.fill_(float("nan"))
    group.Mult(xs, ys)
    for part, yt in zip(parts, ys):
        y[part.owned_global] = host(yt)
    assert relerr(y, ref) <= RTOL


def test_c5_full_size_eight_way_sdirk():
    """configs[4]'s implicit step on its 8-way split: one SDIRK33 step of
    M du/dt = -K u (ode.cpp:834-859, ex16p.cpp:373-470) at 68^3 p = 4 through Operator(group) -- T and
    K as 8-member loopback groups, the group's dots global, Dirichlet dofs held, each stage a
    constrained Jacobi-PCG with a fixed 8 iterations -- against the same step on the serial form (itself
    pinned to oracle/ode.py by test_c5_sdirk_step_full_size)."""
    n, nranks, order, dt, iters = 68, 8, 4, 0.02, 8
    m = E.Mesh.MakeCartesian3D(n, n, n)
    fes = E.H1Space(m, order, E.NUMBERING_STRUCTURED)
    er = E.partition_slabs_z(m, nranks)
    q1d = O.default_q1d(order)
    c = E.ode_implicit_coeff(23)
    a_fn = lambda P: alpha_bioheat(P) / 3.6e6
    b_fn = lambda P: k_of_T(temperature(P))
    ess = fes.boundary_dofs()
    u0 = np.random.default_rng(69).uniform(-1.0, 1.0, fes.ndofs)
    # the serial form's step
    P = O.quad_points(m.element_nodes(), q1d)
    T = _serial_form(fes, None, a_fn(P), c * dt * b_fn(P))
    K = _serial_form(fes, None, None, b_fn(P))
    del P
    u = dev(u0)
    ns, it, conv = E.ode_step(23, E.Operator(T), E.Operator(K), dt, u, ess=dev(ess, torch.int32), rel_tol=0.0,
                              max_iter=iters)
    assert ns == 3 and it == 3 * iters
    us = host(u)
    del T, K, u
    # the group's step
    Tf, parts = _c5_group(m, fes, er, nranks, a_fn, lambda P: c * dt * b_fn(P), q1d)
    Kf, _ = _c5_group(m, fes, er, nranks, None, b_fn, q1d)
    Tg, Kg = E.ParGroup(Tf), E.ParGroup(Kf)
    ug = dev(np.concatenate([u0[p.owned_global] for p in parts]))
    idx, o = [], 0
    for p in parts:
        idx.append(np.nonzero(np.isin(p.owned_global, ess))[0] + o)
        o += p.n_owned
    essg = dev(np.concatenate(idx).astype(np.int32), torch.int32)
    ns, it, conv = E.ode_step(23, E.Operator(Tg), E.Operator(Kg), dt, ug, ess=essg, rel_tol=0.0, max_iter=iters)
    assert ns == 3 and it == 3 * iters
    ugh = host(ug)
    uh = np.empty(fes.ndofs)
    o = 0
    for p in parts:
        uh[p.owned_global] = ugh[o: o + p.n_owned]
        o += p.n_owned
    assert np.array_equal(uh[ess], u0[ess])
    assert relerr(uh - u0, us - u0) < 1e-9


@pytest.mark.parametrize("decomp", ["rap", "overlap"])
def test_c4_eight_way_boxes(decomp):
    """The 2 x 2 x 2 box split of configs[3] (bench.py --partition boxes; SURVEY §8(d) names
    both): up to 7 neighbours per rank (faces, edges, the corner) in the exchange schedule, the
    gathered Mult against the serial oracle."""
    n, nranks, order = 16, 8, 2
    m = E.Mesh.MakeCartesian3D(n, n, n)
    fes = E.H1Space(m, order, E.NUMBERING_STRUCTURED)
    er = E.partition_boxes(m, (2, 2, 2))
    q1d = O.default_q1d(order)
    xg = np.random.default_rng(11).uniform(-1, 1, fes.ndofs)
    forms, parts, xs, ys = [], [], [], []
    for r in range(nranks):
        part = E.Partition(fes, er, r, nranks, decomposition=decomp)
        pf = E.ParBilinearForm(part)
        P = E.quadrature_points_subset(m, q1d, part.elems)
        pf.AddDomainIntegrator(E.MassIntegrator(E.QuadratureCoefficient(dev(alpha_bioheat(P).reshape(part.ne_local, -1)))))
        pf.AddDomainIntegrator(E.DiffusionIntegrator(E.QuadratureCoefficient(
            dev(k_of_T(temperature(P)).reshape(part.ne_local, -1)))))
        pf.Assemble()
        forms.append(pf)
        parts.append(part)
        xs.append(dev(xg[part.owned_global]))
        ys.append(torch.full((part.n_owned,), float("nan"), dtype=torch.float64, device="cuda"))
    assert max(p.n_nbrs for p in parts) == 7
    group = E.ParGroup(forms)
    for _ in range(2):
        group.Mult(xs, ys)
    y = np.full(fes.ndofs, np.nan)
    for part, yt in zip(parts, ys):
        y[part.owned_global] = host(yt)
    Pg = O.quad_points(m.element_nodes(), q1d)
    ref = O.OracleOperator(m.element_nodes(), fes.gather_map(), fes.ndofs, order, alpha=alpha_bioheat(Pg),
                           beta=k_of_T(temperature(Pg))).mult(xg)
    assert relerr(y, ref) <= RTOL


@pytest.mark.parametrize("decomp", ["rap", "overlap"])
def test_slabs_mixed_lattice_addressing(decomp):
    """2-way z-slabs thick enough for complete 4x4x4 blocks: each rank's interior blocks are
    lattice-addressed and its ghost-touching blocks read the map (per-block mode, per-block
    partial-slot layout), the partitioned Mult still matching the serial oracle."""
    nx, nz, nranks, order = 16, 24, 2, 2
    m = E.Mesh.MakeCartesian3D(nx, nx, nz, 1.0, 1.0, nz / nx)
    fes = E.H1Space(m, order, E.NUMBERING_STRUCTURED)
    er = E.partition_slabs_z(m, nranks)
    q1d = O.default_q1d(order)
    xg = np.random.default_rng(9).uniform(-1, 1, fes.ndofs)
    forms, parts, xs, ys, info = [], [], [], [], []
    for r in range(nranks):
        part = E.Partition(fes, er, r, nranks, decomposition=decomp)
        pf = E.ParBilinearForm(part)
        P = E.quadrature_points_subset(m, q1d, part.elems)
        pf.AddDomainIntegrator(E.MassIntegrator(E.QuadratureCoefficient(dev(alpha_bioheat(P).reshape(part.ne_local, -1)))))
        pf.AddDomainIntegrator(E.DiffusionIntegrator(E.QuadratureCoefficient(
            dev(k_of_T(temperature(P)).reshape(part.ne_local, -1)))))
        pf.Assemble()
        info.append(pf.AddressingInfo()[:2])
        forms.append(pf)
        parts.append(part)
        xs.append(dev(xg[part.owned_global]))
        ys.append(torch.full((part.n_owned,), float("nan"), dtype=torch.float64, device="cuda"))
    # every rank lattice-addresses blocks; a rank with ghost dofs also reads the map for some
    # (the lowest rank owns the interface plane: with RAP all its blocks can be regular)
    assert all(lat > 0 for lat, _ in info) and any(lat < units for lat, units in info), info
    group = E.ParGroup(forms)
    group.Mult(xs, ys)
    y = np.full(fes.ndofs, np.nan)
    for part, yt in zip(parts, ys):
        y[part.owned_global] = host(yt)
    Pg = O.quad_points(m.element_nodes(), q1d)
    ref = O.OracleOperator(m.element_nodes(), fes.gather_map(), fes.ndofs, order, alpha=alpha_bioheat(Pg),
                           beta=k_of_T(temperature(Pg))).mult(xg)
    assert relerr(y, ref) <= RTOL
    # the diagonal kernel writes the same per-block slot layouts
    dg = [torch.full((p.n_owned,), float("nan"), dtype=torch.float64, device="cuda") for p in parts]
    group.AssembleDiagonal(dg)
    d = np.full(fes.ndofs, np.nan)
    for part, dt in zip(parts, dg):
        d[part.owned_global] = host(dt)
    dref = O.OracleOperator(m.element_nodes(), fes.gather_map(), fes.ndofs, order, alpha=alpha_bioheat(Pg),
                            beta=k_of_T(temperature(Pg))).diagonal()
    assert relerr(d, dref) <= RTOL


# ---------------------------------------------------------------------------------------
# boundary: MultTranspose / AddMult (bilinearform_ext.hpp:99, operator.hpp:87-92)
# ---------------------------------------------------------------------------------------
@pytest.mark.parametrize("order", [2, 4])
def test_mult_transpose_and_add_mult(order):
    """test_assembly_levels.cpp:96-252 checks MultTranspose PA == legacy; the operator is
    symmetric, so A^T x == A x, and y^T (A x) == x^T (A y)."""
    m = fichera(1)
    fes = E.H1Space(m, order)
    en = m.element_nodes()
    P = O.quad_points(en, O.default_q1d(order))
    a, b = alpha_bioheat(P), coeff_function(P)
    form = _serial_form(fes, P, a, b)
    op = O.OracleOperator(en, fes.gather_map(), fes.ndofs, order, alpha=a, beta=b)
    rng = np.random.default_rng(order)
    x, z = rng.uniform(-1, 1, fes.ndofs), rng.uniform(-1, 1, fes.ndofs)
    yt = torch.full((fes.ndofs,), float("nan"), dtype=torch.float64, device="cuda")
    form.MultTranspose(dev(x), yt)
    ym = torch.empty_like(yt)
    form.Mult(dev(x), ym)
    assert torch.equal(yt, ym)
    assert relerr(host(yt), op.fa_mult(x)) <= RTOL   # legacy (element-matrix) transpose = itself
    zt = torch.empty_like(yt)
    form.MultTranspose(dev(z), zt)
    assert abs(z @ host(yt) - x @ host(zt)) <= 1e-12 * np.abs(z) @ np.abs(host(yt))
    acc = dev(z.copy())
    form.AddMult(dev(x), acc, -0.5)
    assert relerr(host(acc), z - 0.5 * op.mult(x)) <= 1e-12


def test_par_form_mult_transpose_loopback_free():
    """The distributed boundary's MultTranspose (RCCL, one rank) equals its Mult."""
    m = E.Mesh.MakeCartesian3D(4, 3, 6)
    fes = E.H1Space(m, 2)
    part = E.Partition(fes, np.zeros(m.GetNE(), np.int32), 0, 1)
    pf = E.ParBilinearForm(part, rccl_id=E.rccl_unique_id())
    pf.AddDomainIntegrator(E.MassIntegrator(E.ConstantCoefficient(2.0)))
    pf.AddDomainIntegrator(E.DiffusionIntegrator(E.ConstantCoefficient(0.5)))
    pf.Assemble()
    x = dev(np.random.default_rng(3).uniform(-1, 1, part.n_owned))
    y1, y2 = torch.empty_like(x), torch.empty_like(x)
    pf.Mult(x, y1)
    pf.MultTranspose(x, y2)
    assert torch.equal(y1, y2)


# ---------------------------------------------------------------------------------------
# §8(f)1: device Pennes perfusion law for the mass integrator
# ---------------------------------------------------------------------------------------
@pytest.mark.parametrize("order", [2, 4])
def test_perfusion_coefficient(order):
    """alpha(T) = rho c + gamma dt c_b w_b(T) from an H1 temperature field, evaluated on the
    device at Assemble (projection: qfunction.cpp:73-98 restated by the oracle; the law is the
    application's, parity-unpinned) beside the conductivity k(T); Mult and diagonal against the
    oracle with the same laws on the oracle's projection."""
    m = fichera(2) if order == 2 else fichera(1)
    fes = E.H1Space(m, order)
    en = m.element_nodes()
    q1d = O.default_q1d(order)
    T = temperature(fes.dof_coords())            # 37 .. 57 C: the hot spot coagulates
    Tq = BH.temperature_at_quadrature(T, fes.gather_map(), order, q1d)
    # shut-down temperature in the middle of a gap of the quadrature temperatures, so that no
    # point sits on the law's discontinuity (rounding cannot flip a side)
    ts = np.unique(Tq.ravel())
    gaps = np.diff(ts)
    mid = np.argmax(gaps * ((ts[:-1] > 45.0) & (ts[1:] < 55.0)))
    t_stop = 0.5 * (ts[mid] + ts[mid + 1])
    par = (3.6e6, 0.05 * 3.6e3, 6.4e-3, 0.02, 37.0, t_stop)
    ks, kslope, ktref = 0.5 * 0.05, 0.0012, 37.0
    form = E.BilinearForm(fes)
    form.AddDomainIntegrator(E.MassIntegrator(E.PerfusionCoefficient(dev(T), *par)))
    form.AddDomainIntegrator(E.DiffusionIntegrator(E.AffineGridFunctionCoefficient(dev(T), ks, kslope, ktref)))
    form.Assemble()
    alpha = BH.perfusion_law(Tq, *par)
    assert (alpha == par[0]).any() and (alpha > par[0]).any()  # both sides of the shut-down
    beta = BH.affine_law(Tq, ks, kslope, ktref)
    op = O.OracleOperator(en, fes.gather_map(), fes.ndofs, order, alpha=alpha, beta=beta)
    assert relerr(form.qdata(E.MASS)[:, 0, :], op.M) < 1e-13
    x = np.random.default_rng(order).uniform(-1, 1, fes.ndofs)
    y = torch.empty(fes.ndofs, dtype=torch.float64, device="cuda")
    form.Mult(dev(x), y)
    assert relerr(host(y), op.mult(x)) <= RTOL
    d = torch.empty_like(y)
    form.AssembleDiagonal(d)
    assert relerr(host(d), op.diagonal()) < 1e-13


# ---------------------------------------------------------------------------------------
# the distributed form's graph cache across re-assembly (the graphs bake in buffers)
# ---------------------------------------------------------------------------------------
@pytest.mark.parametrize("order", [2, 4])
@pytest.mark.parametrize("schedule", ["serial", "overlap"])
def test_rccl_graph_cache_follows_reassembly(order, schedule):
    m = E.Mesh.MakeCartesian3D(6, 5, 4)
    fes = E.H1Space(m, order)
    part = E.Partition(fes, np.zeros(m.GetNE(), np.int32), 0, 1)
    q1d = O.default_q1d(order)
    P = E.quadrature_points_subset(m, q1d, part.elems)
    c = coeff_function(P).reshape(part.ne_local, -1)
    pf = E.ParBilinearForm(part, rccl_id=E.rccl_unique_id(), schedule=schedule, graph=1)
    pf.AddDomainIntegrator(E.MassIntegrator(E.QuadratureCoefficient(dev(c))))
    pf.AddDomainIntegrator(E.DiffusionIntegrator(E.QuadratureCoefficient(dev(c))))
    pf.Assemble()
    Pg = O.quad_points(m.element_nodes(), q1d)
    cg = coeff_function(Pg)
    ref = O.OracleOperator(m.element_nodes(), fes.gather_map(), fes.ndofs, order, alpha=cg, beta=cg)
    xg = np.random.default_rng(6).uniform(-1, 1, fes.ndofs)
    yref = ref.mult(xg)
    x = dev(xg[part.owned_global])
    y = torch.empty_like(x)

    def check():
        y.fill_(float("nan"))
        for _ in range(3):           # direct, then graph capture, then replay
            pf.Mult(x, y)
        yy = np.zeros(fes.ndofs)
        yy[part.owned_global] = host(y)
        assert relerr(yy, yref) <= RTOL

    check()
    layouts = [pf.info()["layout"]]
    pf.SetGeometryCompression(False)   # frees and reallocates qdata, selects another kernel
    pf.Assemble()
    check()
    layouts.append(pf.info()["layout"])
    assert layouts[0] != layouts[1]
    pf.SetKernel(E.KERNEL_WPE)          # rebuilds the maps and plans
    pf.Assemble()
    check()
    with pytest.raises(E.ECM2Error):   # a setter without Assemble: no stale replay
        pf.SetKernel(E.KERNEL_AUTO)
        pf.Mult(x, y)


# ---------------------------------------------------------------------------------------
# lattice addressing: structured numbering (lattice-addressed kernels) vs entity numbering
# (map-reading kernels), same mesh and coefficients, both against the oracle
# ---------------------------------------------------------------------------------------
@pytest.mark.parametrize("order,n", [(1, 16), (2, 16), (2, 12), (4, 8)])
def test_lattice_addressing_matches_map_path(order, n):
    m = E.Mesh.MakeCartesian3D(n, n, n)
    en = m.element_nodes()
    P = O.quad_points(en, order + 2)
    a, b = alpha_bioheat(P), k_of_T(temperature(P))
    # p = 1: the entity numbering (vertices of MakeCartesian3D) is itself a lattice numbering
    for numbering, lattice in ((E.NUMBERING_STRUCTURED, 1), (E.NUMBERING_ENTITY, 1 if order == 1 else 0)):
        fes = E.H1Space(m, order, numbering)
        form = E.BilinearForm(fes)
        form.AddDomainIntegrator(E.MassIntegrator(quad_coeff(fes, a)))
        form.AddDomainIntegrator(E.DiffusionIntegrator(quad_coeff(fes, b)))
        form.Assemble()
        # n = 12 at p = 2: 1728 elements = 27 full 64-element blocks, lattice-addressed too
        lat, units, _ = form.AddressingInfo()
        assert (lat == units > 0) if lattice else lat == 0, (numbering, form.AddressingInfo())
        op = O.OracleOperator(en, fes.gather_map(), fes.ndofs, order, alpha=a, beta=b)
        x = np.random.default_rng(40 + order).uniform(-1, 1, fes.ndofs)
        y = torch.full((fes.ndofs,), float("nan"), dtype=torch.float64, device="cuda")
        form.Mult(dev(x), y)
        assert relerr(host(y), op.mult(x)) <= RTOL
        d = torch.full((fes.ndofs,), float("nan"), dtype=torch.float64, device="cuda")
        form.AssembleDiagonal(d)
        assert relerr(host(d), op.diagonal()) <= RTOL
