#!/bin/bash
# NOTE: the experiment's switch was deleted with the losing variant after this run; the script is
# kept as the recipe that produced the committed result (profiles/r2_ab_*.txt).
# Round-2 matrix-core experiment at C5 (68^3, p = 4), one box:
#   ECM2_BRICK_MFMA=1: the brick kernel's x stage ([lines x D] x [D x 2Q] per brick) on
#                      v_mfma_f64_16x16x4f64 tiles (k_apply_brick_c<..., MF = true>)
#   default:           the same stage on the VALU (v_fma_f64)
# brick parity tests under the MFMA variant, then bench lines (alternating, twice each) and a
# rocprofv3 kernel-trace of each.
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/ab_mfma
mkdir -p "$O"
export TMPDIR=/tmp
ECM2_BRICK_MFMA=1 timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "brick or c5 or line or sdirk" > "$O/pytest_mfma.log" 2>&1 || { tail -30 "$O/pytest_mfma.log"; exit 1; }
tail -2 "$O/pytest_mfma.log"
for rep in 1 2; do
  for v in 1 0; do
    ECM2_BRICK_MFMA=$v timeout -k 10 300 python3 bench.py --workload c5 --steps 30 --warmup 5 --no-cpu-baseline \
      --full-layout 0 > "$O/bench_v${v}_r${rep}.json" 2> "$O/bench_v${v}_r${rep}.err" || exit $?
    python3 -c "import json,sys; d=json.loads(open('$O/bench_v${v}_r${rep}.json').read().strip().splitlines()[-1]); print('MFMA=$v rep $rep', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_avg'])"
  done
done
for v in 1 0; do
  ECM2_BRICK_MFMA=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace_v$v" -o run --output-format csv \
    -- python3 bench.py --workload c5 --steps 20 --warmup 3 --no-cpu-baseline --full-layout 0 > "$O/trace_v$v.json" 2>&1 || exit $?
  find "$O/trace_v$v" -name "*kernel_stats.csv" -exec head -3 {} \;
done
