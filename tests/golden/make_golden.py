"""Writes tests/golden/oracle_golden.npz: small regression vectors from the CPU oracle.

These are ORACLE-generated (the reference cannot be built here; see DESIGN.md
"Oracle"), used to pin the restatement against accidental change and as fixed
inputs/outputs for the GPU parity tests.  Run: python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
sys.path.insert(0, os.path.join(HERE, ".."))
import oracle as O  # noqa: E402
from helpers import coeff_function, nonaligned  # noqa: E402

out = {}
for order in (1, 2, 3):
    en, gm, nd, xyz = O.cartesian_mesh(2, 2, 2, order=order, transform=nonaligned)
    q1d = O.default_q1d(order)
    P = O.quad_points(en, q1d)
    op = O.OracleOperator(en, gm, nd, order, alpha=coeff_function(P), beta=coeff_function(P))
    x = np.random.default_rng(100 + order).uniform(-1, 1, nd)
    out[f"p{order}_x"] = x
    out[f"p{order}_y"] = op.mult(x)
    out[f"p{order}_diag"] = op.diagonal()
np.savez_compressed(os.path.join(HERE, "oracle_golden.npz"), **out)
print("wrote", sorted(out))
