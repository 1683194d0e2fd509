#!/bin/bash
# per-member plan statistics of the C4 split (lattice-addressed blocks, summation runs) at N = 1, 2, 8
set -uo pipefail
timeout -k 10 300 python3 -c "
import sys; sys.path.insert(0, 'profiles'); import slab_probe, bench, torch
E = bench.load_pkg(); E.load_library()
mesh = E.Mesh.MakeCartesian3D(108, 108, 108, 1.0, 1.0, 1.0)
fes = E.H1Space(mesh, 2, E.NUMBERING_STRUCTURED)
a, T = bench.bioheat_coefficients(E, torch, mesh, fes)
f = E.BilinearForm(fes)
f.AddDomainIntegrator(E.MassIntegrator(E.QuadratureCoefficient(a)))
f.AddDomainIntegrator(E.DiffusionIntegrator(E.AffineGridFunctionCoefficient(T, bench.K_SCALE, bench.K_SLOPE, bench.K_TREF)))
f.Assemble()
print('serial: lattice/units/runs', f.AddressingInfo(), 'shared/slots', f.ScatterInfo(), flush=True)
" || exit $?
for N in 2 8; do timeout -k 10 300 python3 profiles/slab_probe.py members $N || exit $?; done
