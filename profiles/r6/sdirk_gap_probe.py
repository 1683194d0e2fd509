#!/usr/bin/env python3
"""VERDICT r5 item 6, the operator side of the smooth-state SDIRK gap (GPU; profiles/r6/gpu21.sh): at configs[4]
size (68^3, p = 4, 20.3M DoF) the device's K = K_beta applied to the random state, the smooth state
u0 = 37 + 20 exp(-4 |x - 1/2|^2) and the shifted state u0 - 37, against the oracle's K in the mesh's element
order, and the oracle's K with its elements permuted against the same -- the norm of each product's difference.  A product
of a smooth state cancels (K 1 = 0, and the smooth part is a Laplacian times h^3), so its rounding relative
to |K u| is what 8 unconverged PCG iterations then amplify.  Then the smooth state's SDIRK33 step with 8 fixed
iterations per stage through two device forms that round differently -- the default compressed geometry (the
brick kernel on AFFINE_E) and the per-point layout (SetGeometryCompression(False)) -- against each other and
against the oracle's step (tests/golden/sdirk_c5_smooth_fixed8.npz).  Test infrastructure: the oracle is the
checker."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import oracle as O  # noqa: E402
from helpers import alpha_bioheat, k_of_T, relerr, temperature  # noqa: E402

sys.path.insert(0, ROOT)
import __graft_entry__ as G  # noqa: E402

E = G._load_pkg()
E.load_library()


def main():
    n, order = 68, 4
    m = E.Mesh.MakeCartesian3D(n, n, n)
    fes = E.H1Space(m, order, E.NUMBERING_STRUCTURED)
    en, gm = m.element_nodes(), fes.gather_map()
    P = O.quad_points(en, O.default_q1d(order))
    alpha, beta = alpha_bioheat(P) / 3.6e6, k_of_T(temperature(P))
    del P
    K = E.BilinearForm(fes)
    K.AddDomainIntegrator(E.DiffusionIntegrator(E.QuadratureCoefficient(
        torch.from_numpy(np.ascontiguousarray(beta.reshape(fes.ne, -1))).cuda())))
    K.Assemble()
    X = fes.dof_coords()
    smooth = 37.0 + 20.0 * np.exp(-4.0 * np.sum((X - 0.5) ** 2, axis=1))
    states = {"random": np.random.default_rng(68).uniform(-1.0, 1.0, fes.ndofs), "smooth": smooth,
              "shifted": smooth - 37.0, "constant 37": np.full(fes.ndofs, 37.0)}
    Kr = O.OracleOperator(en, gm, fes.ndofs, order, beta=beta)
    perm = np.random.default_rng(7).permutation(fes.ne)
    Kp = O.OracleOperator(en[perm], gm[perm], fes.ndofs, order, beta=beta[perm])
    print(f"# configs[4] K_beta, {fes.ndofs} DoF; relerr against the oracle's K u (mesh element order)", flush=True)
    for name, u in states.items():
        y = torch.empty(fes.ndofs, dtype=torch.float64, device="cuda")
        K.Mult(torch.from_numpy(u).cuda(), y)
        yd = y.cpu().numpy()
        yr, yp = Kr.mult(u), Kp.mult(u)
        print(f"{name:12s} |u|_2 = {np.linalg.norm(u):.4e}  |K u|_2 oracle {np.linalg.norm(yr):.4e} device "
              f"{np.linalg.norm(yd):.4e} permuted {np.linalg.norm(yp):.4e}   |K u - K_oracle u|_2 device "
              f"{np.linalg.norm(yd - yr):.3e} permuted {np.linalg.norm(yp - yr):.3e}", flush=True)
    del K, Kr, Kp
    sdirk_forms(fes, alpha, beta, fes.boundary_dofs(), smooth)


def sdirk_forms(fes, alpha, beta, ess, u0):
    dt = 0.02
    c = E.ode_implicit_coeff(23)
    g = np.load(os.path.join(ROOT, "tests", "golden", "sdirk_c5_smooth_fixed8.npz"))
    idx = g["idx"]

    def qc(v):
        return E.QuadratureCoefficient(torch.from_numpy(np.ascontiguousarray(v.reshape(fes.ne, -1))).cuda())

    du = {}
    for name, compress in (("compressed geometry", True), ("per-point geometry", False)):
        T, K = E.BilinearForm(fes), E.BilinearForm(fes)
        for f in (T, K):
            f.SetGeometryCompression(compress)
        T.AddDomainIntegrator(E.MassIntegrator(qc(alpha)))
        T.AddDomainIntegrator(E.DiffusionIntegrator(qc(c * dt * beta)))
        K.AddDomainIntegrator(E.DiffusionIntegrator(qc(beta)))
        T.Assemble()
        K.Assemble()
        u = torch.from_numpy(u0.copy()).cuda()
        ns, it, conv = E.ode_step(23, E.Operator(T), E.Operator(K), dt, u, ess=torch.from_numpy(ess).to(torch.int32).cuda(),
                                  rel_tol=0.0, max_iter=8)
        du[name] = u.cpu().numpy() - u0
        print(f"device SDIRK33 step, fixed 8, {name:20s} (kernel {T.info()['kernel']}, layout {T.info()['layout']}): "
              f"iterations {it}; relerr against the oracle's step {relerr(du[name][idx], g['u1'] - g['u0']):.3e}",
              flush=True)
        del T, K, u
    a, b = du.values()
    print(f"relerr between the two device forms' steps: {relerr(b, a):.3e}", flush=True)


if __name__ == "__main__":
    main()
