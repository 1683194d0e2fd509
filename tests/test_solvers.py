"""The callers of the PA operator: constrained Jacobi-PCG on the
serial form, on the partitioned form (loopback group on one GPU; the RCCL rank path runs
the same solver with ncclAllReduce'd dots), and the implicit ODE steps of an ex16-style
conduction operator (BackwardEuler / SDIRK23 / SDIRK33 / ImplicitMidpoint / SDIRK34,
ode.cpp:682-859).

CPU tests pin the oracle's ODE restatement (oracle/ode.py) on y' = -lam*y; GPU tests
compare the device solvers with the oracle's PCG and stepping on the same inputs."""
import math

import numpy as np
import pytest

import helpers  # noqa: F401
import ecm2_amd as E
import oracle as O
import ode as ODE
from helpers import GOLDEN, coeff_function, nonaligned, relerr

TYPES = [21, 22, 23, 32, 33, 34]
ORDER = {21: 1, 22: 2, 23: 3, 32: 2, 33: 3, 34: 4}


# ---------------------------------------------------------------------------------------
# CPU: the oracle's ODE restatement and the library's stage coefficients
# ---------------------------------------------------------------------------------------
@pytest.mark.parametrize("ode_type", TYPES)
def test_ode_oracle_order_of_convergence(ode_type):
    """y' = -lam y: (1 + c dt lam) k = -lam u is the stage solve; the global error falls
    with the method's order (ode.cpp tableau comments)."""
    lam, T = 1.3, 1.0
    c = ODE.implicit_coeff(ode_type)
    errs = []
    for n in (20, 40, 80):
        dt = T / n
        solve = lambda u: -lam * u / (1.0 + c * dt * lam)
        u = np.array([1.0])
        for _ in range(n):
            u = ODE.step(ode_type, solve, u, dt)
        errs.append(abs(u[0] - math.exp(-lam * T)))
    rate = math.log2(errs[1] / errs[2])
    assert abs(rate - ORDER[ode_type]) < 0.25, (ode_type, errs, rate)


@pytest.mark.parametrize("ode_type", TYPES)
def test_ode_implicit_coeff_matches_oracle(ode_type):
    assert E.ode_implicit_coeff(ode_type) == pytest.approx(ODE.implicit_coeff(ode_type), rel=1e-15)
    with pytest.raises(E.ECM2Error):
        E.ode_implicit_coeff(99)


# ---------------------------------------------------------------------------------------
# GPU
# ---------------------------------------------------------------------------------------
def _mesh(kind):
    if kind == "cart":
        m = E.Mesh.MakeCartesian3D(5, 4, 6)
        m.set_vertices(nonaligned(m.vertices()))
        return m
    m = E.Mesh(f"{GOLDEN}/fichera.mesh")
    m.UniformRefinement()
    return m


def _elem_rank(m, kind, nranks):
    if kind == "cart":
        return E.partition_slabs_z(m, nranks)
    return np.random.default_rng(5).integers(0, nranks, m.GetNE()).astype(np.int32)


def _alpha(P):
    return 2.0 + np.sin(P[..., 0]) * np.cos(P[..., 1])


def _beta(P):
    return coeff_function(P)


def _group(m, fes, order, er, nranks, alpha_fn, beta_fn, scale_beta=1.0):
    import torch
    q1d = O.default_q1d(order)
    forms, parts = [], []
    for r in range(nranks):
        part = E.Partition(fes, er, r, nranks)
        pf = E.ParBilinearForm(part)
        P = E.quadrature_points_subset(m, q1d, part.elems)
        if alpha_fn is not None:
            pf.AddDomainIntegrator(E.MassIntegrator(E.QuadratureCoefficient(
                torch.as_tensor(alpha_fn(P).reshape(part.ne_local, -1)).cuda())))
        if beta_fn is not None:
            pf.AddDomainIntegrator(E.DiffusionIntegrator(E.QuadratureCoefficient(
                torch.as_tensor(scale_beta * beta_fn(P).reshape(part.ne_local, -1)).cuda())))
        pf.Assemble()
        forms.append(pf)
        parts.append(part)
    return E.ParGroup(forms), parts


def _serial(m, fes, order, alpha_fn, beta_fn, scale_beta=1.0):
    import torch
    q1d = O.default_q1d(order)
    P = O.quad_points(m.element_nodes(), q1d)
    f = E.BilinearForm(fes)
    if alpha_fn is not None:
        f.AddDomainIntegrator(E.MassIntegrator(E.QuadratureCoefficient(
            torch.as_tensor(alpha_fn(P).reshape(fes.ne, -1)).cuda())))
    if beta_fn is not None:
        f.AddDomainIntegrator(E.DiffusionIntegrator(E.QuadratureCoefficient(
            torch.as_tensor(scale_beta * beta_fn(P).reshape(fes.ne, -1)).cuda())))
    f.Assemble()
    return f


def _oracle(m, fes, order, alpha_fn, beta_fn, scale_beta=1.0):
    q1d = O.default_q1d(order)
    P = O.quad_points(m.element_nodes(), q1d)
    a = alpha_fn(P) if alpha_fn is not None else None
    b = scale_beta * beta_fn(P) if beta_fn is not None else None
    return O.OracleOperator(m.element_nodes(), fes.gather_map(), fes.ndofs, order, alpha=a, beta=b)


def _to_group(vec_global, parts):
    return np.concatenate([vec_global[p.owned_global] for p in parts])


def _from_group(vec_group, parts, n):
    out = np.zeros(n)
    o = 0
    for p in parts:
        out[p.owned_global] = vec_group[o: o + p.n_owned]
        o += p.n_owned
    return out


def _group_ess(ess_global, parts):
    """Global essential dofs -> indices in the group's concatenated true vector."""
    idx, o = [], 0
    for p in parts:
        pos = np.nonzero(np.isin(p.owned_global, ess_global))[0]
        idx.append(pos + o)
        o += p.n_owned
    return np.concatenate(idx).astype(np.int32)


@pytest.mark.gpu
@pytest.mark.parametrize("kind,nranks", [("cart", 2), ("cart", 3), ("fichera", 3), ("fichera", 4)])
def test_group_diagonal_matches_oracle(kind, nranks):
    import torch
    m = _mesh(kind)
    fes = E.H1Space(m, 2)
    er = _elem_rank(m, kind, nranks)
    group, parts = _group(m, fes, 2, er, nranks, _alpha, _beta)
    ds = [torch.empty(p.n_owned, dtype=torch.float64, device="cuda") for p in parts]
    group.AssembleDiagonal(ds)
    d = _from_group(np.concatenate([x.cpu().numpy() for x in ds]), parts, fes.ndofs)
    assert relerr(d, _oracle(m, fes, 2, _alpha, _beta).diagonal()) < 1e-13


@pytest.mark.gpu
@pytest.mark.parametrize("kind,nranks", [("cart", 1), ("cart", 3), ("fichera", 4)])
@pytest.mark.parametrize("jacobi", [True, False])
def test_group_pcg_matches_oracle(kind, nranks, jacobi):
    """Partitioned constrained PCG (dots over the group = global dots) == serial oracle PCG."""
    import torch
    m = _mesh(kind)
    fes = E.H1Space(m, 2)
    er = _elem_rank(m, kind, nranks)
    group, parts = _group(m, fes, 2, er, nranks, _alpha, _beta)
    op = E.Operator(group)
    assert op.size == fes.ndofs
    ess = fes.boundary_dofs()
    b = np.random.default_rng(4).uniform(-1, 1, fes.ndofs)
    x = torch.empty(fes.ndofs, dtype=torch.float64, device="cuda")
    it, _ = op.PCG(torch.as_tensor(_to_group(b, parts)).cuda(), x,
                   ess=torch.as_tensor(_group_ess(ess, parts)).cuda(), rel_tol=1e-12, max_iter=2000, jacobi=jacobi)
    xr, itr, _ = _oracle(m, fes, 2, _alpha, _beta).pcg(b, ess, rel_tol=1e-12, max_iter=2000, jacobi=jacobi)
    assert abs(it - itr) <= 2
    assert relerr(_from_group(x.cpu().numpy(), parts, fes.ndofs), xr) < 1e-9


@pytest.mark.gpu
@pytest.mark.parametrize("ode_type", TYPES)
def test_ode_step_matches_oracle(ode_type):
    """Two implicit steps of M du/dt = -K u with Dirichlet boundary dofs held fixed: device
    ode_step on the serial form == oracle stepping with the oracle's PCG stage solves."""
    import torch
    m = _mesh("cart")
    order = 2
    fes = E.H1Space(m, order)
    dt = 0.05
    c = E.ode_implicit_coeff(ode_type)
    T = _serial(m, fes, order, _alpha, _beta, scale_beta=c * dt)
    K = _serial(m, fes, order, None, _beta)
    Tr = _oracle(m, fes, order, _alpha, _beta, scale_beta=c * dt)
    Kr = _oracle(m, fes, order, None, _beta)
    ess = fes.boundary_dofs()
    X = fes.dof_coords()
    u0 = 37.0 + 20.0 * np.exp(-4.0 * np.sum((X - 0.5) ** 2, axis=1))

    def solve(us):
        rhs = -Kr.mult(us)
        rhs[ess] = 0.0
        return Tr.pcg(rhs, ess, rel_tol=1e-13, max_iter=5000)[0]

    ur = u0.copy()
    for _ in range(2):
        ur = ODE.step(ode_type, solve, ur, dt)
    u = torch.as_tensor(u0).cuda()
    essd = torch.as_tensor(ess).cuda()
    for _ in range(2):
        ns, it, conv = E.ode_step(ode_type, E.Operator(T), E.Operator(K), dt, u, ess=essd, rel_tol=1e-13,
                                  max_iter=5000)
        assert conv and ns == {21: 1, 32: 1, 22: 2, 33: 2, 23: 3, 34: 3}[ode_type]
    uh = u.cpu().numpy()
    assert np.array_equal(uh[ess], u0[ess])
    assert relerr(uh - u0, ur - u0) < 1e-9


@pytest.mark.gpu
@pytest.mark.parametrize("kind,nranks", [("cart", 3), ("fichera", 4)])
def test_ode_step_group_matches_serial(kind, nranks):
    """SDIRK33 on the partitioned operators (loopback group) == the serial device step."""
    import torch
    m = _mesh(kind)
    order = 2
    fes = E.H1Space(m, order)
    dt, ode_type = 0.02, 23
    c = E.ode_implicit_coeff(ode_type)
    er = _elem_rank(m, kind, nranks)
    Tg, parts = _group(m, fes, order, er, nranks, _alpha, _beta, scale_beta=c * dt)
    Kg, _ = _group(m, fes, order, er, nranks, None, _beta)
    Ts = _serial(m, fes, order, _alpha, _beta, scale_beta=c * dt)
    Ks = _serial(m, fes, order, None, _beta)
    ess = fes.boundary_dofs()
    u0 = np.random.default_rng(3).uniform(30, 40, fes.ndofs)
    us = torch.as_tensor(u0).cuda()
    E.ode_step(ode_type, E.Operator(Ts), E.Operator(Ks), dt, us, ess=torch.as_tensor(ess).cuda(), rel_tol=1e-13,
               max_iter=5000)
    ug = torch.as_tensor(_to_group(u0, parts)).cuda()
    E.ode_step(ode_type, E.Operator(Tg), E.Operator(Kg), dt, ug,
               ess=torch.as_tensor(_group_ess(ess, parts)).cuda(), rel_tol=1e-13, max_iter=5000)
    ugh = _from_group(ug.cpu().numpy(), parts, fes.ndofs)
    assert relerr(ugh - u0, us.cpu().numpy() - u0) < 1e-9
