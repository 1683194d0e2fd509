#!/bin/bash
# Round 4: SQ counters at this round's tree for the drop-in configuration (TRILINEAR lattice kernel,
# reference numbering + Jacobians) and C5 (brick kernel + summation pass), the counters the verdict
# asked for beside the PMC pins.
set -uo pipefail
export TMPDIR=/tmp
bash profiles/sq_pass.sh r4_dropin --workload c4 --numbering entity --mesh trilinear --geometry-input jacobians --variants 0 --full-layout 0 --steps 20 --warmup 3 > /dev/null 2>&1 || exit 1
bash profiles/sq_pass.sh r4_c5 --workload c5 --variants 0 --full-layout 0 --steps 20 --warmup 3 > /dev/null 2>&1 || exit 1
SQ_COUNTERS="SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_ANY" \
  bash profiles/sq_pass.sh r4_c5b --workload c5 --variants 0 --full-layout 0 --steps 20 --warmup 3 > /dev/null 2>&1 || exit 1
python3 - <<'PY'
import json, os
root = os.environ.get("GRAFT_REPO_ROOT", ".")
for tag in ("r4_dropin", "r4_c5", "r4_c5b"):
    d = json.load(open(f"{root}/gpurun_out/sq_{tag}/sq_summary.json"))
    for k, v in d.items():
        if "apply" in k or "sum_partials" in k:
            print(tag, k[:40], {a: (round(b, 3) if isinstance(b, float) else b) for a, b in v.items()
                                if a.endswith("frac") or a in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "vgpr")})
PY
