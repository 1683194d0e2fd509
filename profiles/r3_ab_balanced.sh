#!/bin/bash
# Member-mode bench test (interleaved passes, median per member), then a same-box A/B of the N = 8 slab
# partition: CartesianPartitioning's 13 / 14-layer slabs against equal-count slabs (13.5 layers, the
# split layer divided along y; ECM2_SLABS=balanced), emulated per-rank Mult, twice each.
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/balanced
mkdir -p "$O"
timeout -k 10 300 python3 -u -m pytest tests/test_bench.py -m gpu -x -q --timeout 200 --timeout-method thread > "$O/pytest_bench.log" 2>&1
rc=$?; tail -2 "$O/pytest_bench.log"; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in cart balanced; do
    S=""; [ $v = balanced ] && S=balanced
    ECM2_SLABS=$S timeout -k 10 400 python3 bench.py --workload c4 --loopback 8 --member -1 --steps 50 --warmup 5 \
      --no-cpu-baseline --full-layout 0 --variants 0 > "$O/${v}_$rep.json" 2> "$O/${v}_$rep.err" || { tail -5 "$O/${v}_$rep.err"; exit 1; }
    python3 -c "import json,sys; b=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'slowest', b['slowest_member_ms'], 'ms', b['member_ms'], b['member_passes_ms'])" "$O/${v}_$rep.json" "$v rep $rep"
  done
done
