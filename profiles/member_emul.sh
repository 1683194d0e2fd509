#!/bin/bash
# Emulated per-rank Mult of the partitioned C4 operator (bench.py --loopback N --member -1): each
# member's rows alone on the GPU, replayed from a HIP graph, with the stages, streams and kernels
# one RCCL rank runs (exchange as device copies).  The slowest member sets the emulated N-GPU rate.
# Usage: bash profiles/member_emul.sh [N ...]     (default 2 4 8); EXTRA= extra bench flags; LIB= another build
# of the library (run through profiles/ab_lib.py)
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/member
mkdir -p "$O"
WL=${WL:-c4}
RUN="python3 bench.py"
[ -n "${LIB:-}" ] && RUN="python3 profiles/ab_lib.py $LIB"
timeout -k 10 300 $RUN --workload $WL --steps 50 --warmup 5 --no-cpu-baseline --full-layout 0 ${EXTRA:-} \
  > "$O/${WL}${TAG:-}_n1.json" 2> "$O/${WL}${TAG:-}_n1.err" || exit $?
python3 -c "import json,sys; b=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('N=1', b['value'], 'MDoF/s', b['ms_per_step'], 'ms', 'pcg_iteration_ms', (b.get('pcg_iteration') or {}).get('iteration_ms'))" "$O/${WL}${TAG:-}_n1.json"
for N in ${@:-2 4 8}; do
  timeout -k 10 400 $RUN --workload $WL --loopback $N --member -1 --steps 50 --warmup 5 \
    --no-cpu-baseline --full-layout 0 ${EXTRA:-} > "$O/${WL}${TAG:-}_n$N.json" 2> "$O/${WL}${TAG:-}_n$N.err" || exit $?
  python3 -c "import json,sys; b=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); p=b.get('pcg') or {}; print('N=%d' % b['emulated_n_gpus'], b['emulated_value'], 'MDoF/s', 'slowest', b['slowest_member_ms'], 'ms', 'members', b['member_ms'], 'pcg slowest', p.get('slowest_member_iteration_ms'), 'ms/iter', p.get('member_iteration_ms'))" "$O/${WL}${TAG:-}_n$N.json"
done
