#!/bin/bash
# Round 4: TRILINEAR prefetch-depth A/B (r4_ab_pfd.sh), the snapshot kernel's LDS pair layout, then SQ counters of the k(T)-snapshot kernel
# (C4 headline configuration).
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r4sq
mkdir -p "$O"
export TMPDIR=/tmp
bash profiles/r4_ab_pfd.sh || exit $?
# the k(T)-snapshot kernel with (x, T') pairs per lattice slot (tspl: one 16-byte LDS read per point)
bash profiles/ab_libs.sh tspl_c4 "libecm2pa.so libecm2pa_tspl.so" --workload c4 --steps 30 --warmup 5 --variants 0 || exit $?
SQ_COUNTERS="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
  bash profiles/sq_pass.sh c4_ts --workload c4 --variants 0 --full-layout 0 --steps 20 --warmup 3 > "$O/sq_c4ts.txt" 2>&1 || exit 1
python3 - "$O/sq_c4ts.txt" <<'PY'
import json,sys
t=open(sys.argv[1]).read(); d=json.loads(t[t.index('{'):])
for k,v in d.items():
    if 'tpe' in k: print(k, {a:(round(b,3) if isinstance(b,float) else b) for a,b in v.items() if a.endswith('frac') or a in ('SQ_INSTS_VALU','SQ_INSTS_LDS','SQ_LDS_BANK_CONFLICT','vgpr')})
PY
