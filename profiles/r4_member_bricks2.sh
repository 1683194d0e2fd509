#!/bin/bash
# Round 4: brick-run partitions with the snapshot on mixed regular / lattice-map forms (RAP ranks
# ordered as one segment): the distributed GPU tests, then the emulated per-rank Mult at N = 8 / 4 / 2
# for OVERLAP z-slabs (the default) and RAP brick runs, one box.
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r4mb2
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_distributed.py \
  tests/test_gpu_parity.py -k "not test_gpu_parity.py or snapshot" > "$O/tests.txt" 2>&1 || { tail -40 "$O/tests.txt"; exit 1; }
tail -1 "$O/tests.txt"
show() { python3 -c "import json,sys; b=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'N=%d' % b['emulated_n_gpus'], 'slowest', b['slowest_member_ms'], 'members', b['member_ms'], 'snapshot', b.get('coefficient_snapshot'))" "$1" "$2"; }
timeout -k 10 300 python3 bench.py --workload c4 --steps 50 --warmup 5 --no-cpu-baseline --full-layout 0 --variants 0 > "$O/n1.json" 2> "$O/n1.err" || exit 1
python3 -c "import json,sys; b=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('N=1', b['value'], 'MDoF/s', b['ms_per_step'], 'ms')" "$O/n1.json"
for N in 8 4 2; do
  for cfg in "overlap slabs" "rap bricks"; do
    set -- $cfg
    ECM2_DECOMP=$1 timeout -k 10 400 python3 bench.py --workload c4 --loopback $N --member -1 --partition $2 --steps 50 --warmup 5 \
      --no-cpu-baseline --full-layout 0 > "$O/n${N}_$1_$2.json" 2> "$O/n${N}_$1_$2.err" || exit 1
    show "$O/n${N}_$1_$2.json" "$1/$2"
  done
done
