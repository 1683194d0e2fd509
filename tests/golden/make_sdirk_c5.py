"""Writes tests/golden/sdirk_c5_smooth.npz: the oracle's converged SDIRK33 step at configs[4]'s size.

ORACLE-generated golden values (the reference cannot be built here; see DESIGN.md "Oracle"): one
SDIRK33 step (oracle/ode.py, ode.cpp:834-859) of M du/dt = -K u on Cartesian 68^3 at p = 4
(20,346,417 DoF, the structured numbering), alpha = rho c_eff / 3.6e6, beta = k(T), dt = 0.02, the
boundary dofs held, from the SMOOTH state u0 = 37 + 20 exp(-4 |x - 1/2|^2), every stage a constrained
Jacobi-PCG solved to rel_tol 1e-12 (oracle/pa_oracle.c orc_pcg).  The whole vector is 163 MB, so the
fixture keeps u1 at 20,000 seeded random dofs plus u1's norms; tests/test_gpu_configs.py::
test_c5_sdirk_smooth_converged compares the device step there.  The oracle
takes ~45 min on 8 threads: run python tests/golden/make_sdirk_c5.py in this container, not in a test.
"""
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests"), ROOT]
import oracle as O  # noqa: E402
import ode as ODE  # noqa: E402
from helpers import alpha_bioheat, k_of_T, temperature  # noqa: E402
import __graft_entry__ as G  # noqa: E402

N, ORDER, DT, NSAMPLE = 68, 4, 0.02, 20000


def smooth_state(X):
    return 37.0 + 20.0 * np.exp(-4.0 * np.sum((X - 0.5) ** 2, axis=1))


def main():
    E = G._load_pkg()
    E.load_library()
    m = E.Mesh.MakeCartesian3D(N, N, N)
    fes = E.H1Space(m, ORDER, E.NUMBERING_STRUCTURED)
    en, gm = m.element_nodes(), fes.gather_map()
    P = O.quad_points(en, O.default_q1d(ORDER))
    alpha, beta = alpha_bioheat(P) / 3.6e6, k_of_T(temperature(P))
    del P
    c = ODE.implicit_coeff(23)
    Tr = O.OracleOperator(en, gm, fes.ndofs, ORDER, alpha=alpha, beta=c * DT * beta)
    Kr = O.OracleOperator(en, gm, fes.ndofs, ORDER, beta=beta)
    ess = fes.boundary_dofs()
    u0 = smooth_state(fes.dof_coords())
    its = []

    def solve(us):
        rhs = -Kr.mult(us)
        rhs[ess] = 0.0
        xs, it, _ = Tr.pcg(rhs, ess, rel_tol=1e-12, max_iter=100000)
        assert Tr.last_pcg_status == 1
        its.append(it)
        return xs

    t0 = time.time()
    u1 = ODE.step(23, solve, u0, DT)
    idx = np.sort(np.random.default_rng(2026).choice(fes.ndofs, NSAMPLE, replace=False)).astype(np.int64)
    np.savez_compressed(os.path.join(HERE, "sdirk_c5_smooth.npz"), idx=idx, u1=u1[idx], u0=u0[idx],
                        du_norm2=np.linalg.norm(u1 - u0), du_max=np.abs(u1 - u0).max(), iterations=np.array(its),
                        ndofs=np.array(fes.ndofs))
    print(f"wrote sdirk_c5_smooth.npz: stage iterations {its}, |u1 - u0|_inf {np.abs(u1 - u0).max():.6e}, "
          f"{time.time() - t0:.0f} s")


if __name__ == "__main__":
    main()
