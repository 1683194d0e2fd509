#!/usr/bin/env python3
"""Kernel time of one rank-sized slab of C4 on one GPU (a serial form on a 108 x 108 x nz Cartesian
mesh, the same coefficients as bench.py): how the per-rank interior kernel of an N-way z-slab
split scales with the slab's thickness (whole 4 x 4 x 4 brick layers or leftover layers, number of
workgroups against the 512 that fit at once).
Usage: python3 profiles/slab_probe.py nz [nz ...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    import torch
    E = bench.load_pkg()
    E.load_library()
    for nz in [int(a) for a in sys.argv[1:]]:
        mesh = E.Mesh.MakeCartesian3D(108, 108, nz, 1.0, 1.0, nz / 108)
        fes = E.H1Space(mesh, 2, E.NUMBERING_STRUCTURED)
        a, T = bench.bioheat_coefficients(E, torch, mesh, fes)
        f = E.BilinearForm(fes)
        f.AddDomainIntegrator(E.MassIntegrator(E.QuadratureCoefficient(a)))
        f.AddDomainIntegrator(E.DiffusionIntegrator(E.AffineGridFunctionCoefficient(T, bench.K_SCALE, bench.K_SLOPE, bench.K_TREF)))
        f.Assemble()
        x = torch.empty(fes.ndofs, dtype=torch.float64, device="cuda").uniform_(-1, 1)
        y = torch.empty_like(x)
        kms = bench.kernel_ms([f], f.Mult, x, y, 100, torch)
        dt = bench.time_mults(f.Mult, x, y, 100, 5, 1, None, torch)
        lat, units, runs = f.AddressingInfo()
        nsh, nslots = f.ScatterInfo()
        print(f"nz={nz:3d} elements {fes.ne:7d} blocks {(fes.ne + 63) // 64:5d} workgroups {(fes.ne + 255) // 256:5d} "
              f"lattice-addressed {lat}/{units} shared {nsh} runs {runs}  kernel {kms * 1e3:6.1f} us  Mult {dt / 100 * 1e6:6.1f} us  "
              f"per element {kms * 1e6 / fes.ne:.3f} ns", flush=True)
        del f, a, T, x, y
        torch.cuda.synchronize()


def members(N):
    """The N z-slab members of C4 (loopback partition, as bench.py --loopback N builds them):
    local elements, lattice-addressed blocks, summation-plan runs."""
    import torch
    E = bench.load_pkg()
    E.load_library()
    mesh = E.Mesh.MakeCartesian3D(108, 108, 108, 1.0, 1.0, 1.0)
    fes = E.H1Space(mesh, 2, E.NUMBERING_STRUCTURED)
    er = E.partition_slabs_z(mesh, N)
    keep = []
    for r in range(N):
        part = E.Partition(fes, er, r, N)
        pf = E.ParBilinearForm(part)
        a, T = bench.bioheat_coefficients(E, torch, mesh, fes, part)
        pf.AddDomainIntegrator(E.MassIntegrator(E.QuadratureCoefficient(a)))
        pf.AddDomainIntegrator(E.DiffusionIntegrator(E.AffineGridFunctionCoefficient(T, bench.K_SCALE, bench.K_SLOPE, bench.K_TREF)))
        pf.Assemble()
        lat, units, runs = pf.AddressingInfo()
        print(f"member {r}/{N}: local elements {part.ne_local} owned {part.ne_owned} lattice-addressed {lat}/{units} "
              f"runs {runs}", flush=True)
        keep += [pf, part, a, T]


if __name__ == "__main__":
    if sys.argv[1] == "members":
        members(int(sys.argv[2]))
    else:
        main()
