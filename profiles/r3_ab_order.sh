#!/bin/bash
# A/B (same box): face-linked bricks along a Morton curve of their cells (c) vs in the caller's
# element order (f) -- C4 with the reference's numbering (SFC element order) and C3 fichera
set -uo pipefail
bash profiles/ab_libs.sh ord_c4e "libecm2pa_c.so libecm2pa_f.so" --workload c4 --steps 50 --warmup 5 --variants 0 --numbering entity || exit $?
bash profiles/ab_libs.sh ord_c3 "libecm2pa_c.so libecm2pa_f.so" --workload c3 --steps 30 --warmup 5 || exit $?
