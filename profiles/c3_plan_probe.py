import os, sys
sys.path.insert(0, os.getcwd())
import bench
import torch
E = bench.load_pkg(); E.load_library()
for ref in (5, 6):
    mesh = E.Mesh(os.path.join(os.getcwd(), "tests", "golden", "fichera.mesh"))
    for _ in range(ref): mesh.UniformRefinement()
    fes = E.H1Space(mesh, 2)
    a, T = bench.bioheat_coefficients(E, torch, mesh, fes)
    f = E.BilinearForm(fes)
    f.AddDomainIntegrator(E.MassIntegrator(E.QuadratureCoefficient(a)))
    f.AddDomainIntegrator(E.DiffusionIntegrator(E.AffineGridFunctionCoefficient(T, bench.K_SCALE, bench.K_SLOPE, bench.K_TREF)))
    f.Assemble()
    print("refine", ref, "ndofs", fes.ndofs, "ne", fes.ne, "scatter (shared, slots)", f.ScatterInfo(), "addressing (lattice, units, runs)", f.AddressingInfo(), flush=True)
