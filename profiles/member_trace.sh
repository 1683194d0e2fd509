#!/bin/bash
# Kernel timeline of one member's graph-replayed Mult (bench.py --loopback N --member R) under
# rocprofv3 --kernel-trace.  Usage: bash profiles/member_trace.sh N R [N R ...]
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/member_trace
mkdir -p "$O"
export TMPDIR=/tmp
while [ $# -ge 2 ]; do
  N=$1; R=$2; shift 2
  T=${WL:-c4}${TAG:-}-n$N-m$R
  timeout -k 10 300 rocprofv3 --kernel-trace -d "$O/$T" -o run --output-format csv \
    -- python3 bench.py --workload ${WL:-c4} --loopback $N --member $R --steps 30 --warmup 5 --no-cpu-baseline \
    --full-layout 0 ${EXTRA:-} > "$O/$T.json" 2> "$O/$T.err" || exit $?
  echo "== N=$N member $R: $(python3 -c "import json,sys; b=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(b['member_ms'])" "$O/$T.json") ms"
  python3 profiles/member_trace.py "$O/$T" 3 || exit $?
done
