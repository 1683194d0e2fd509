#!/bin/bash
# Round 4: the k(T) snapshot on mixed forms (lattice bricks + element-map blocks with a stored W beta:
# a partitioned rank's local form) -- parity on the GPU, then the emulated per-rank Mult against the
# stored-pair path (nomix: ECM2_TSNAP_MIXED=0), same box, interleaved.
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r4tsmix
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_distributed.py tests/test_gpu_configs.py tests/test_gpu_parity.py \
  -k "loopback or snapshot or marker or eight_way or slabs_mixed or member or rccl or gridfunction or perfusion or c3" > "$O/tests.txt" 2>&1 || { tail -40 "$O/tests.txt"; exit 1; }
tail -1 "$O/tests.txt"
for rep in 1 2; do
  for v in libecm2pa.so libecm2pa_nomix.so; do
    for N in 2 8; do
      timeout -k 10 400 python3 profiles/ab_lib.py cardiac-ablation-ecm2_amd/lib/$v --workload c4 --loopback $N --member -1 \
        --steps 50 --warmup 5 --no-cpu-baseline --full-layout 0 > "$O/${v}_n${N}_$rep.json" 2> "$O/${v}_n${N}_$rep.err" || { tail -20 "$O/${v}_n${N}_$rep.err"; exit 1; }
      python3 -c "import json,sys; b=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('$v N=$N rep $rep', b['emulated_value'], 'slowest', b['slowest_member_ms'], 'members', b['member_ms'])" "$O/${v}_n${N}_$rep.json"
    done
  done
done
