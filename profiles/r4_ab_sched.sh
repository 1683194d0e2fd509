#!/bin/bash
# Round 4: the p = 2 kernels under LLVM's alternative AMDGPU scheduler strategies (k_tpe.hip built with
# -mllvm -amdgpu-sched-strategy=max-ilp / iterative-ilp; everything else identical): C4 (snapshot
# kernel), then the trilinear mesh (max-ilp only: iterative-ilp spills 55 values there).
set -uo pipefail
export TMPDIR=/tmp
bash profiles/ab_libs.sh sched_c4 "libecm2pa.so libecm2pa_smaxilp.so libecm2pa_siterativeilp.so" --workload c4 --steps 30 --warmup 5 --variants 0 || exit $?
bash profiles/ab_libs.sh sched_c4t "libecm2pa.so libecm2pa_smaxilp.so" --workload c4 --mesh trilinear --steps 30 --warmup 5 --variants 0 || exit $?
