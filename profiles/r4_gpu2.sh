#!/bin/bash
# Round 4: TRILINEAR_E (p >= 3) and p >= 3 diffusion-only layouts on the GPU, the full-size drop-in
# test, then the pending A/Bs (r4_ab_pf2.sh) and a C5 bench line with its trilinear sub-object.
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r4g2
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "trilinear_e or diffusion_only or jacobian_geometry or affine_geometry or reference_numbering or attribute_markers" \
  > "$O/tests.txt" 2>&1 || { tail -30 "$O/tests.txt"; exit 1; }
tail -2 "$O/tests.txt"
timeout -k 10 300 python -u bench.py --workload c5 --steps 20 --warmup 3 > "$O/bench_c5.json" 2> "$O/bench_c5.err" || { tail -20 "$O/bench_c5.err"; exit 1; }
python - "$O/bench_c5.json" <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("c5", d["value"], d["ms_per_step"], d["roofline"].get("kernel_ms_avg"))
for k in ("full_layout","entity_numbering","trilinear","drop_in"):
    if k in d: print(k, d[k].get("value"), d[k].get("ms_per_step"), d[k].get("qdata_layout"), d[k]["roofline"].get("kernel_ms_avg"))
PY
bash profiles/r4_ab_pf2.sh
