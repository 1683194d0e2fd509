#!/bin/bash
# The driver's default bench line at this tree (C4 + full_layout / entity_numbering / trilinear), C5, C3
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r3default
mkdir -p "$O"
timeout -k 10 500 python3 bench.py > "$O/bench_c4.json" 2> "$O/bench_c4.err" || exit $?
python3 - "$O/bench_c4.json" <<'PY'
import json, sys
b = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = b["roofline"]
print("c4", b["value"], b["ms_per_step"], r["kernel_ms_avg"], r["frac"], b["config"]["lattice_units"], b["config"]["summation_runs"])
for k in ("full_layout", "entity_numbering", "trilinear"):
    d = b[k]; r = d["roofline"]
    print(k, d["value"], d["ms_per_step"], r["kernel_ms_avg"], r["alg_ratio"], d["qdata_layout"], d["lattice_units"], d["summation_runs"], d["plan"])
print(b["cpu_baseline"])
PY
timeout -k 10 500 python3 bench.py --workload c5 --steps 30 --warmup 5 --no-cpu-baseline --full-layout 0 > "$O/bench_c5.json" 2> "$O/bench_c5.err" || exit $?
tail -1 "$O/bench_c5.json" | cut -c1-300
