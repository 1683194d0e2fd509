#!/usr/bin/env python3
"""Diagnostic: the summation plan's run classes (ECM2_PLAN_DUMP) for the structured and the
reference numbering at a given Cartesian size."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["ECM2_PLAN_DUMP"] = "1"
import bench  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 24
import torch  # noqa: E402
E = bench.load_pkg()
E.load_library()
for numbering in ("structured", "entity"):
    mesh, fes = bench.cartesian_space(E, n, n, n, 2, numbering, "affine")
    f = E.BilinearForm(fes)
    f.AddDomainIntegrator(E.MassIntegrator(E.ConstantCoefficient(2.0)))
    f.AddDomainIntegrator(E.DiffusionIntegrator(E.ConstantCoefficient(1.0)))
    print(numbering, flush=True)
    sys.stderr.flush()
    f.Assemble()
    torch.cuda.synchronize()
    print(numbering, "plan info", f.PlanInfo(), f.AddressingInfo(), f.ScatterInfo(), flush=True)
