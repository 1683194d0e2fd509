#!/bin/bash
# Round 4: TRILINEAR lattice kernel, rows of point values in flight (PFD) x per-plane z partials (ZP):
# p11 = one row + partials (the committed form), p21 = two rows + partials (29 values spilled),
# p20 = two rows + per-row lattice re-read (256 VGPRs, no spills); pNOPAIR = no point-value loads
# (timing probe: the bound). C4 trilinear mesh, then the drop-in configuration.
set -uo pipefail
export TMPDIR=/tmp
L="libecm2pa_p11.so libecm2pa_p21.so libecm2pa_p20.so libecm2pa_pnp.so"
bash profiles/ab_libs.sh pfd_c4t "$L" --workload c4 --steps 30 --warmup 5 --variants 0 --mesh trilinear || exit $?
bash profiles/ab_libs.sh pfd_c4d "libecm2pa_p11.so libecm2pa_p21.so libecm2pa_p20.so" --workload c4 --steps 30 --warmup 5 --variants 0 --mesh trilinear --numbering entity --geometry-input jacobians || exit $?
