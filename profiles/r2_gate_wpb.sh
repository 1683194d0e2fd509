#!/bin/bash
# (Needs the WPB experiment code, measured and removed: profiles/r2_ab_wpb.txt; kept as the record of the run.)
# two waves per block (k_apply_tpe_sf WPB = 2) for small launches: suite (auto), then A/B by ECM2_TPE_WPB
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/wpb
mkdir -p "$O"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
rc=$?
tail -2 "$O/pytest_gpu.log"; grep -E "FAILED|ERROR" "$O/pytest_gpu.log" | head -20
[ $rc -eq 0 ] || exit $rc
for N in 8 4 2; do for W in 1 2 1 2; do
  ECM2_TPE_WPB=$W timeout -k 10 300 python3 bench.py --loopback $N --member -1 --steps 50 --warmup 5 --no-cpu-baseline --full-layout 0 > $O/m$N-w$W.json 2> $O/m$N-w$W.err || exit $?
  python3 -c "import json; d=json.loads(open('$O/m$N-w$W.json').read().strip().splitlines()[-1]); print('N=$N wpb=$W', d['slowest_member_ms'], d['member_ms'])"
done; done
for WL in c2 c4; do for W in 1 2; do
  ECM2_TPE_WPB=$W timeout -k 10 300 python3 bench.py --workload $WL --steps 50 --warmup 5 --no-cpu-baseline --full-layout 0 > $O/$WL-w$W.json 2> $O/$WL-w$W.err || exit $?
  python3 -c "import json; d=json.loads(open('$O/$WL-w$W.json').read().strip().splitlines()[-1]); print('$WL wpb=$W', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_avg'])"
done; done
