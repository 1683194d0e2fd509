#!/bin/bash
# Round 4: where the TRILINEAR lattice kernel waits -- timing probes (wrong results, timing only):
# no point-value loads (pNOPAIR), no x gather (pNOGATHER) against the real kernel, C4 trilinear mesh;
# then the default bench line (drop_in sub-object with the per-plane-partials kernel).
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r4tlp
mkdir -p "$O"
export TMPDIR=/tmp
bash profiles/ab_libs.sh tlprobe_c4t "libecm2pa.so libecm2pa_pNOPAIR.so libecm2pa_pNOGATHER.so" --workload c4 --steps 30 --warmup 5 --variants 0 --mesh trilinear || exit $?
timeout -k 10 400 python -u bench.py > "$O/bench.json" 2> "$O/bench.err" || { tail -20 "$O/bench.err"; exit 1; }
python - "$O/bench.json" <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("c4", d["value"], d["ms_per_step"], d["roofline"].get("kernel_ms_avg"), d["roofline"].get("frac"))
for k in ("full_layout","entity_numbering","trilinear","drop_in"):
    if k in d: print(k, d[k].get("value"), d[k].get("ms_per_step"), d[k].get("qdata_layout"), d[k]["roofline"].get("kernel_ms_avg"))
PY
