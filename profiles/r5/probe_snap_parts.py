"""Probe (round 5): which partitioned forms take the k(T) coefficient snapshot -- per rank, for the
z-slab and brick-run splits of test_distributed.py::test_gpu_loopback_group_coefficient_snapshot."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np
import torch
import helpers  # noqa: F401  (registers ecm2_amd)
import ecm2_amd as E
from helpers import temperature

E.load_library()
for split in ("slabs", "bricks"):
    for decomp in ("rap", "overlap"):
        m = E.Mesh.MakeCartesian3D(8, 8, 8) if split == "slabs" else E.Mesh.MakeCartesian3D(12, 8, 8)
        fes = E.H1Space(m, 2)
        nr = 2 if split == "slabs" else 3
        er = E.partition_slabs_z(m, 2) if split == "slabs" else E.partition_bricks(m, 3)
        T = temperature(fes.dof_coords())
        out = []
        for r in range(nr):
            part = E.Partition(fes, er, r, nr, decomposition=decomp)
            pf = E.ParBilinearForm(part)
            Tl = torch.as_tensor(T[part.local_to_global]).cuda()
            pf.AddDomainIntegrator(E.MassIntegrator(E.ConstantCoefficient(1.0)))
            pf.AddDomainIntegrator(E.DiffusionIntegrator(E.AffineGridFunctionCoefficient(Tl, 0.05, 0.0012, 37.0)))
            pf.Assemble()
            out.append((bool(pf.CoefficientSnapshot()), pf.AddressingInfo()[:2], part.ne_local, part.n_ghost))
        print(split, decomp, out, flush=True)
