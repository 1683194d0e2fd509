#!/bin/bash
# Round 4: GPU suite at the tree, then same-box A/B of the TRILINEAR kernels on the trilinear C4 mesh
# (structured numbering: RM 1) and the drop-in configuration (reference numbering + MFEM Jacobians: RM 3):
# tlold = per-element kernel (with the (W beta / det J, W alpha det J) pairs), tlA = lattice kernel,
# rows refilled per point, tlB = lattice kernel, ping-pong rows.
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r4tlb
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
rc=$?
tail -3 "$O/pytest_gpu.log"; grep -E "FAILED|ERROR" "$O/pytest_gpu.log" | head -20
[ $rc -eq 0 ] || exit $rc
bash profiles/ab_libs.sh tlb_c4t "libecm2pa_tlold.so libecm2pa_tlA.so libecm2pa_tlB.so" --workload c4 --steps 30 --warmup 5 --variants 0 --mesh trilinear || exit $?
bash profiles/ab_libs.sh tlb_drop "libecm2pa_tlold.so libecm2pa_tlA.so libecm2pa_tlB.so" --workload c4 --steps 30 --warmup 5 --variants 0 --mesh trilinear --numbering entity --geometry-input jacobians || exit $?
# C5 brick kernel: in-wave stage hand-offs without workgroup barriers (brws) against the tree before it (tlA)
bash profiles/ab_libs.sh brws_c5 "libecm2pa_tlA.so libecm2pa_brws.so" --workload c5 --steps 30 --warmup 5 --variants 0 || exit $?
