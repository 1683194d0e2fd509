#!/usr/bin/env python3
"""Where does the reference-numbering gap at C4 come from?  Same box, same mesh (the reference's
MakeCartesian3D with its space-filling-curve element order), the same operator under dof
renumberings of the reference's FiniteElementSpace numbering (the form only sees the gather map):

  structured  lexicographic elements + lattice numbering (the headline)
  entity      the reference's numbering (vertices, edges, faces, interiors; first-insertion order)
  classlex    entity numbering, each entity class (8 lattice parity classes) renumbered in
              lexicographic order of its points: a piecewise lattice with the same class blocks
  brickfirst  entity numbering renumbered in order of first touch by the kernel's bricks: the
              best locality any numbering can give this processing order

Every variant's y is mapped back to the entity numbering and compared with the entity result.
Usage: python3 profiles/r3_numbering_probe.py [--n 108] [--steps 100] [--rounds 2]"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


class Renumbered:
    """An H1 space whose dofs are renumbered by newid (old dof -> new dof)."""

    def __init__(self, fes, newid):
        self._f, self.newid = fes, newid
        self.mesh, self.ne, self.order, self.ndofs, self.nd = fes.mesh, fes.ne, fes.order, fes.ndofs, fes.nd

    def gather_map(self):
        g = self._f.gather_map()
        neg = g < 0
        out = self.newid[np.where(neg, -1 - g, g)]
        return np.where(neg, -1 - out, out).astype(np.int32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=108)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--check-only", action="store_true")
    a = ap.parse_args()
    import torch
    E = bench.load_pkg()
    E.load_library()
    n = a.n
    spaces = {}
    ms, fs = bench.cartesian_space(E, n, n, n, 2, "structured", "affine")
    me, fe = bench.cartesian_space(E, n, n, n, 2, "entity", "affine")
    # lattice position of every entity dof (p = 2: 2n + 1 points per direction)
    X = np.rint(fe.dof_coords() * (2 * n)).astype(np.int64)
    cls = (X[:, 0] & 1) + 2 * (X[:, 1] & 1) + 4 * (X[:, 2] & 1)
    lex = (X[:, 2] * (2 * n + 1) + X[:, 1]) * (2 * n + 1) + X[:, 0]
    order = np.lexsort((lex, cls))
    newid = np.empty(fe.ndofs, np.int64)
    newid[order] = np.arange(fe.ndofs)
    spaces["classlex"] = (me, Renumbered(fe, newid))
    # first touch in the kernel's element order (the brick order the form uses on this mesh)
    perm = me.element_order(E.ORDER_BRICK)
    g = fe.gather_map()[perm].ravel()
    _, first = np.unique(g, return_index=True)
    nb = np.empty(fe.ndofs, np.int64)
    nb[np.unique(g)[np.argsort(first)]] = np.arange(fe.ndofs)
    spaces["brickfirst"] = (me, Renumbered(fe, nb))
    spaces["entity"] = (me, fe)
    spaces["structured"] = (ms, fs)
    # the entity space's dof -> structured dof (coordinates)
    Xs = np.rint(fs.dof_coords() * (2 * n)).astype(np.int64)
    lex_s = (Xs[:, 2] * (2 * n + 1) + Xs[:, 1]) * (2 * n + 1) + Xs[:, 0]
    to_s = np.full((2 * n + 1) ** 3, -1, np.int64)
    to_s[lex_s] = np.arange(fs.ndofs)
    maps = {"entity": np.arange(fe.ndofs), "classlex": newid, "brickfirst": nb, "structured": to_s[lex]}
    for v, m in maps.items():
        assert np.array_equal(np.sort(m), np.arange(fe.ndofs)), v
    # the renumbered gather maps are the entity map through the permutation
    ge, gs = fe.gather_map(), fs.gather_map()
    assert np.array_equal(spaces["classlex"][1].gather_map(), newid[ge])
    if a.check_only:
        print("maps ok", fe.ndofs)
        return
    # maps[v][d_entity] = the variant's dof for entity dof d
    xe = np.random.default_rng(5).uniform(-1, 1, fe.ndofs)
    Te = 37.0 + np.random.default_rng(6).uniform(0, 20, fe.ndofs)
    forms, xs, ys = {}, {}, {}
    for v, (mesh, sp) in spaces.items():
        m = maps[v]
        T = np.empty(fe.ndofs)
        T[m] = Te
        Tt = torch.tensor(T, device="cuda")
        f = E.BilinearForm(sp)
        f.AddDomainIntegrator(E.MassIntegrator(E.ConstantCoefficient(3.7e6)))
        f.AddDomainIntegrator(E.DiffusionIntegrator(E.AffineGridFunctionCoefficient(Tt, bench.K_SCALE, bench.K_SLOPE,
                                                                                     bench.K_TREF)))
        f.Assemble()
        f._T = Tt
        xv = np.empty(fe.ndofs)
        xv[m] = xe
        forms[v] = f
        xs[v] = torch.tensor(xv, device="cuda")
        ys[v] = torch.empty_like(xs[v])
        info = {"variant": v, "layout": f.info().get("layout"), "plan": f.PlanInfo(), "scatter": f.ScatterInfo()}
        print(json.dumps(info, default=str), flush=True)
    ref = None
    for r in range(a.rounds):
        for v, f in forms.items():
            kms = bench.kernel_ms([f], f.Mult, xs[v], ys[v], a.steps, torch)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.steps):
                f.Mult(xs[v], ys[v])
            e1.record()
            torch.cuda.synchronize()
            mult = e0.elapsed_time(e1) / a.steps
            y = ys[v].cpu().numpy()[maps[v]]
            if ref is None:
                ref = y
            err = float(np.abs(y - ref).max() / np.abs(ref).max())
            print(json.dumps({"variant": v, "round": r, "mult_ms": round(mult, 5), "kernel_ms": round(kms, 5),
                              "rest_ms": round(mult - kms, 5), "MDoF_s": round(fe.ndofs / mult / 1e3, 1),
                              "relerr_vs_first": err}), flush=True)


if __name__ == "__main__":
    main()
