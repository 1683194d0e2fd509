#!/bin/bash
# Round 4 gate: the whole -m gpu suite, smoke(), then the default bench line (N = 1), on one box.
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r4gate
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > "$O/gpu_tests.txt" 2>&1 || { tail -40 "$O/gpu_tests.txt"; exit 1; }
tail -2 "$O/gpu_tests.txt"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.txt" 2>&1 || { tail -20 "$O/smoke.txt"; exit 1; }
tail -1 "$O/smoke.txt"
timeout -k 10 600 python -u bench.py > "$O/bench.json" 2> "$O/bench.err" || { tail -20 "$O/bench.err"; exit 1; }
python3 - "$O/bench.json" <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r=d["roofline"]
print("c4", d["value"], d["ms_per_step"], r.get("kernel_ms_avg"), r.get("frac"), r.get("alg_ratio"), d["config"].get("qdata_layout"))
for k in ("full_layout","entity_numbering","trilinear","drop_in"):
    if k in d: print(k, d[k].get("value"), d[k].get("ms_per_step"), d[k].get("qdata_layout"), d[k]["roofline"].get("kernel_ms_avg"))
print("cpu", d.get("cpu_baseline"))
PY
