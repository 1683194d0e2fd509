#!/bin/bash
# round 3: GPU suite at the working tree, then the default bench line (C4 + full-layout,
# entity-numbering and trilinear sub-objects) and C3
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r3bench
mkdir -p "$O"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
rc=$?
tail -3 "$O/pytest_gpu.log"; grep -E "FAILED|ERROR" "$O/pytest_gpu.log" | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python3 bench.py --cpu-baseline-seconds 5 > "$O/bench_c4.json" 2> "$O/bench_c4.err" || exit $?
python3 - "$O/bench_c4.json" <<'PY'
import json, sys
b = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
def show(tag, d):
    r = d["roofline"]
    print(tag, d["value"], d["ms_per_step"], r["kernel_ms_avg"], d.get("qdata_layout", d.get("config", {}).get("qdata_layout")),
          d.get("lattice_units", d.get("config", {}).get("lattice_units")), d.get("summation_runs", d.get("config", {}).get("summation_runs")))
show("c4", b)
for k in ("full_layout", "entity_numbering", "trilinear"):
    if k in b: show(k, b[k])
PY
timeout -k 10 500 python3 bench.py --workload c3 --steps 30 --warmup 5 --no-cpu-baseline > "$O/bench_c3.json" 2> "$O/bench_c3.err" || exit $?
tail -1 "$O/bench_c3.json" | cut -c1-600
