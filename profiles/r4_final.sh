#!/bin/bash
# Round-4 close: the gate (whole -m gpu suite, smoke, default bench line) at HEAD, then the SQ pass of
# the drop-in configuration after the TRILINEAR kernel's coefficient reload.
set -uo pipefail
export TMPDIR=/tmp
bash profiles/r4_gate.sh || exit 1
bash profiles/sq_pass.sh r4_dropin2 --workload c4 --numbering entity --mesh trilinear --geometry-input jacobians --variants 0 --full-layout 0 --steps 20 --warmup 3 > /dev/null 2>&1 || exit 1
python3 - <<'PY'
import json, os
d = json.load(open(os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out/sq_r4_dropin2/sq_summary.json")))
v = d["k_apply_tpe_tlb"]
print("tlb", {k: (round(x, 3) if isinstance(x, float) and x < 10 else x) for k, x in v.items()})
PY
