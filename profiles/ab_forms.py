#!/usr/bin/env python3
"""Same-box A/B of BilinearForm variants on one workload: each variant is assembled once, then
the variants are timed alternately (rounds x), each after a 60 ms settle, as ms per Mult
(HIP events around the timed Mults) and the form's own dominant-kernel event time.
Usage: python3 profiles/ab_forms.py c5 'bricks=1' 'bricks=2' [--rounds 2] [--steps 100]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("workload", choices=["c2", "c4", "c5"])
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--steps", type=int, default=100)
    a = ap.parse_args()
    import torch
    E = bench.load_pkg()
    E.load_library()
    n, order = {"c2": (50, 2), "c4": (108, 2), "c5": (68, 4)}[a.workload]
    mesh = E.Mesh.MakeCartesian3D(n, n, n, 1.0, 1.0, 1.0)
    fes = E.H1Space(mesh, order, E.NUMBERING_STRUCTURED)
    al, T = bench.bioheat_coefficients(E, torch, mesh, fes)
    forms = {}
    for v in a.variants:
        kw = {}
        for item in v.split(","):
            if item:
                k, val = item.split("=")
                kw[k] = int(val) if val.lstrip("-").isdigit() else val
        f = E.BilinearForm(fes, **kw)
        f.AddDomainIntegrator(E.MassIntegrator(E.QuadratureCoefficient(al)))
        f.AddDomainIntegrator(E.DiffusionIntegrator(E.AffineGridFunctionCoefficient(T, bench.K_SCALE, bench.K_SLOPE,
                                                                                    bench.K_TREF)))
        f.Assemble()
        forms[v] = f
    x = torch.empty(fes.ndofs, dtype=torch.float64, device="cuda").uniform_(-1, 1)
    y = torch.empty_like(x)
    ref = None
    out = {"workload": a.workload, "ndofs": fes.ndofs, "runs": []}
    for r in range(a.rounds):
        for v, f in forms.items():
            kms = bench.kernel_ms([f], f.Mult, x, y, a.steps, torch)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.steps):
                f.Mult(x, y)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / a.steps
            if ref is None:
                ref = y.clone()
            err = float((y - ref).abs().max() / ref.abs().max())
            out["runs"].append({"variant": v, "round": r, "mult_ms": round(ms, 5), "kernel_ms": round(kms, 5),
                                "info": f.info() if hasattr(f, "info") else None, "rel_diff_vs_first": err,
                                "MDoF_s": round(fes.ndofs / ms / 1e3, 1)})
            print(json.dumps(out["runs"][-1]), file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
