#!/bin/bash
# Round 4: the snapshot on a split L-vector (loopback group test), then the emulated per-rank Mult
# at N = 2 / 4 / 8 (profiles/member_emul.sh: OVERLAP z-slabs, serial schedule, each member's rows
# alone on the GPU, median of interleaved passes), at this round's tree.
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r4member
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_distributed.py \
  -k "coefficient_snapshot or loopback_group_matches_serial" > "$O/tests.txt" 2>&1 || { tail -40 "$O/tests.txt"; exit 1; }
tail -1 "$O/tests.txt"
bash profiles/member_emul.sh 2 4 8 || exit $?
# the TRILINEAR_E brick kernel built for 3 waves per SIMD (140 VGPRs, no spills) against 4 (128 VGPRs,
# 8 values spilled), C5 trilinear mesh
bash profiles/ab_libs.sh bw3_c5t "libecm2pa.so libecm2pa_bw3.so" --workload c5 --mesh trilinear --steps 30 --warmup 5 --variants 0 || exit $?
