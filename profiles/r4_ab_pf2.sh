#!/bin/bash
# Round 4: the full per-point layout kernel at two waves per SIMD (pf2: one row buffer refilled per
# point, 1D tables instead of the row-product table) against the round-start kernel (tlA's), same box;
# then SQ counters of the lattice TRILINEAR kernel (c4tri) with the LDS counters.
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r4pf2
mkdir -p "$O"
export TMPDIR=/tmp
bash profiles/ab_libs.sh pf2_c4full "libecm2pa_tlA.so libecm2pa_pf2.so" --workload c4 --steps 30 --warmup 5 --variants 0 --geometry full || exit $?
SQ_COUNTERS="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
  bash profiles/sq_pass.sh c4tri_tlb --workload c4 --mesh trilinear --variants 0 --full-layout 0 --steps 20 --warmup 3 > "$O/sq_c4tri.txt" 2>&1 || exit 1
SQ_COUNTERS="SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_ANY" \
  bash profiles/sq_pass.sh c4tri_tlb2 --workload c4 --mesh trilinear --variants 0 --full-layout 0 --steps 20 --warmup 3 > "$O/sq_c4tri2.txt" 2>&1 || exit 1
echo done
# the lattice TRILINEAR kernel with per-plane z partials (tlZ, 2 scratch ops per plane) against per-row (main)
bash profiles/ab_libs.sh tlz_c4t "libecm2pa.so libecm2pa_tlZ.so" --workload c4 --steps 30 --warmup 5 --variants 0 --mesh trilinear || exit $?
