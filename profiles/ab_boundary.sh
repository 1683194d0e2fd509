#!/bin/bash
# Emulated ranks of the weak-scaled C2 partition (graph-captured Mult): boundary elements with
# the plane-per-wave latency kernel (ECM2_BOUNDARY_PP=1, default) or the throughput kernel.
set -eu
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
pr() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], d['value'], 'MDoF/s', d['ms_per_step'], 'ms/step', r['kernel_ms_avg'], 'kernel ms')" "$1" "$2"; }
timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > "$O/bd_n1.json"; pr "$O/bd_n1.json" "N=1"
for pp in 1 0; do
for rw in ${RANKS:-3:8 0:8 1:2}; do
  r=${rw%%:*}; n=${rw##*:}
  ECM2_BOUNDARY_PP=$pp timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --emulate-rank $r --emulate-world $n > "$O/bd_${pp}_${r}_${n}.json"
  pr "$O/bd_${pp}_${r}_${n}.json" "rank $r/$n boundary_pp=$pp"
done
done
