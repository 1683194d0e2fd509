#!/bin/bash
# Emulated ranks (OVERLAP, graph): boundary kernel = plane-per-wave latency kernel or the
# throughput kernel (ECM2_BOUNDARY_PP 1 / 0).
set -eu
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
pr() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], 'MDoF/s', d['ms_per_step'], 'ms/step')" "$1" "$2"; }
timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > "$O/bp_n1.json"; pr "$O/bp_n1.json" "N=1"
timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --graph 1 > "$O/bp_n1g.json"; pr "$O/bp_n1g.json" "N=1 graph"
for pp in 0 1; do
for rw in ${RANKS:-3:8 0:8}; do
  r=${rw%%:*}; n=${rw##*:}
  ECM2_BOUNDARY_PP=$pp timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --emulate-rank $r --emulate-world $n > "$O/bp_${pp}_${r}_${n}.json"
  pr "$O/bp_${pp}_${r}_${n}.json" "rank $r/$n boundary_pp=$pp"
done
done
