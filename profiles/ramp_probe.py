#!/usr/bin/env python3
"""Per-Mult durations of the C4 (or C5) operator from the first Mult after idle onwards, to
see how long the GPU takes to reach its sustained rate (and whether a short idle resets it).
Usage: python3 profiles/ramp_probe.py [c4|c5] > gpurun_out/ramp.json"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main(w):
    import torch
    E = bench.load_pkg()
    E.load_library()
    n, order = (108, 2) if w == "c4" else (68, 4)
    mesh = E.Mesh.MakeCartesian3D(n, n, n, 1.0, 1.0, 1.0)
    fes = E.H1Space(mesh, order, E.NUMBERING_STRUCTURED)
    a, T = bench.bioheat_coefficients(E, torch, mesh, fes)
    f = E.BilinearForm(fes)
    f.AddDomainIntegrator(E.MassIntegrator(E.QuadratureCoefficient(a)))
    f.AddDomainIntegrator(E.DiffusionIntegrator(E.AffineGridFunctionCoefficient(T, bench.K_SCALE, bench.K_SLOPE,
                                                                                bench.K_TREF)))
    f.Assemble()
    x = torch.empty(fes.ndofs, dtype=torch.float64, device="cuda").uniform_(-1, 1)
    y = torch.empty_like(x)
    torch.cuda.synchronize()
    time.sleep(0.5)

    def run(k):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(k + 1)]
        ev[0].record()
        for i in range(k):
            f.Mult(x, y)
            ev[i + 1].record()
        torch.cuda.synchronize()
        return [round(ev[i].elapsed_time(ev[i + 1]) * 1e3, 1) for i in range(k)]

    out = {"workload": w, "ndofs": fes.ndofs}
    out["after_idle_500ms"] = run(200)
    time.sleep(0.005)
    out["after_idle_5ms"] = run(60)
    time.sleep(0.05)
    out["after_idle_50ms"] = run(60)
    print(json.dumps(out))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "c4")
