"""Lattice-addressed block counts of the C4 z-slab local forms at N = 2, 4, 8 (profiles/r2_addr_probe.txt)."""
import sys, json
sys.path.insert(0, '.')
import bench, torch
E = bench.load_pkg(); E.load_library()
n = 108
mesh = E.Mesh.MakeCartesian3D(n, n, n, 1.0, 1.0, 1.0)
fes = E.H1Space(mesh, 2, E.NUMBERING_STRUCTURED)
for nsub in (2, 4, 8):
    er = E.partition_slabs_z(mesh, nsub)
    for r in sorted({0, nsub // 2, nsub - 1}):
        part = E.Partition(fes, er, r, nsub, decomposition="overlap")
        pf = E.ParBilinearForm(part)
        a, T = bench.bioheat_coefficients(E, torch, mesh, fes, part)
        pf.AddDomainIntegrator(E.MassIntegrator(E.QuadratureCoefficient(a)))
        pf.AddDomainIntegrator(E.DiffusionIntegrator(E.AffineGridFunctionCoefficient(T, 0.1, 0.001, 37.0)))
        pf.Assemble()
        print(nsub, r, part.ne_local, part.ne_interior if hasattr(part, 'ne_interior') else None, pf.AddressingInfo(), flush=True)
        del pf
