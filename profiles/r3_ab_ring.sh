#!/bin/bash
# Same-box A/B of the partial-slot order inside each face group: b = [face points lexicographic, edges inline];
# c = bricks (p >= 3) list a face's interior first, then its ring; d = the same for the p <= 2 blocks.
# Parity first: the GPU parity and config suites with c and with d as the library, then timings.
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/ring
mkdir -p "$O"
L=cardiac-ablation-ecm2_amd/lib
for v in c d; do
  cp $L/libecm2pa_$v.so $L/libecm2pa.so
  timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 200 \
    --timeout-method thread > "$O/pytest_$v.log" 2>&1
  rc=$?; echo "$v: $(tail -1 "$O/pytest_$v.log")"
  cp $L/libecm2pa_b.so $L/libecm2pa.so
  [ $rc -eq 0 ] || { grep -E "FAILED|Error" "$O/pytest_$v.log" | head; exit $rc; }
done
bash profiles/ab_libs.sh ring_c5 "libecm2pa_b.so libecm2pa_c.so" --workload c5 --steps 50 --warmup 5 || exit $?
bash profiles/ab_libs.sh ring_c4 "libecm2pa_b.so libecm2pa_d.so" --workload c4 --steps 50 --warmup 5 --variants 0 || exit $?
bash profiles/ab_libs.sh ring_c4e "libecm2pa_b.so libecm2pa_d.so" --workload c4 --numbering entity --steps 50 --warmup 5 --variants 0 || exit $?
bash profiles/ab_libs.sh ring_c3 "libecm2pa_b.so libecm2pa_d.so" --workload c3 --steps 30 --warmup 5 || exit $?
