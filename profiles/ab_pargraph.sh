#!/bin/bash
# Emulated middle rank (3 of 8) of the weak-scaled C2 partition: graph-captured Mult
# (ECM2_PAR_GRAPH 1 / 0) x interior split (ECM2_INTERIOR_SPLIT percent in part A), against N=1.
set -eu
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
pr() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], d['value'], 'MDoF/s', d['ms_per_step'], 'ms/step', r['kernel_ms_avg'], 'kernel ms')" "$1" "$2"; }
timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > "$O/pg_n1.json"; pr "$O/pg_n1.json" "N=1"
for g in ${GRAPHS:-1 0}; do
for sp in ${SPLITS:-50 25 0}; do
  ECM2_PAR_GRAPH=$g ECM2_INTERIOR_SPLIT=$sp timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --emulate-rank ${RANK:-3} --emulate-world ${WORLD:-8} > "$O/pg_${g}_${sp}.json"
  pr "$O/pg_${g}_${sp}.json" "rank ${RANK:-3}/${WORLD:-8} graph=$g split=$sp"
done
done
