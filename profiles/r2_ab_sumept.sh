#!/bin/bash
# (experiment, source not kept in the tree) plan blocks of up to 4 x 256 entries (ECM2_SUM_EPT=4)
# against one entry per thread (ECM2_SUM_EPT=1, the plan in the tree):
# parity first, then C4 / C5 bench lines and the emulated 8-rank C4 member Mult, alternating.
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/sumept
mkdir -p "$O"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_distributed.py tests/test_gpu_configs.py tests/test_solvers.py \
  -m gpu -x -q --timeout 200 --timeout-method thread -k "not full_size" > "$O/parity.log" 2>&1 || { tail -30 "$O/parity.log"; exit 1; }
tail -1 "$O/parity.log"
for E in 1 4 1 4; do
  for WL in c4 c5; do
    ECM2_SUM_EPT=$E timeout -k 10 300 python3 bench.py --workload $WL --steps 50 --warmup 5 --no-cpu-baseline --full-layout 0 \
      > "$O/${WL}_e$E.json" 2> "$O/${WL}_e$E.err" || exit $?
    python3 -c "import json,sys; b=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('EPT=$E $WL', b['value'], 'MDoF/s', b['ms_per_step'], 'ms, kernel', b['roofline']['kernel_ms_avg'], 'ms')" "$O/${WL}_e$E.json"
  done
  ECM2_SUM_EPT=$E TAG=_e$E bash profiles/member_emul.sh 8 2>&1 | tail -1 | sed "s/^/EPT=$E member /" || exit 1
done
