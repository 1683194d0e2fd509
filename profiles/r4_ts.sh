#!/bin/bash
# Round 4: the k(T) coefficient snapshot (k_apply_tpe_ts) -- parity on the GPU, then a same-box A/B
# against the stored W beta (same library, --coefficient-snapshot 1 / 0) on C4 (headline config) and
# with the reference's numbering; then the TRILINEAR prefetch-depth A/B (r4_ab_pfd.sh).
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r4ts
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "coefficient_snapshot or gridfunction or full_size_c4_tpe or rejected_duplicate or attribute_markers" \
  > "$O/tests.txt" 2>&1 || { tail -40 "$O/tests.txt"; exit 1; }
tail -2 "$O/tests.txt"
for rep in 1 2; do
  for ts in 1 0; do
    for num in structured entity; do
      timeout -k 10 300 python3 bench.py --workload c4 --steps 30 --warmup 5 --variants 0 --full-layout 0 --no-cpu-baseline \
        --numbering $num --coefficient-snapshot $ts > "$O/c4_${num}_ts${ts}_$rep.json" 2> "$O/c4_${num}_ts${ts}_$rep.err" || { tail -20 "$O/c4_${num}_ts${ts}_$rep.err"; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/c4_${num}_ts${ts}_$rep.json').read().strip().splitlines()[-1]); print('$num ts$ts rep $rep', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_avg'], d['config'].get('qdata_layout'))"
    done
  done
done
bash profiles/r4_ab_pfd.sh
