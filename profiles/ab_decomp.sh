#!/bin/bash
# Emulated ranks of the weak-scaled C2 partition (graph-captured Mult): OVERLAP decomposition
# (ghost elements, one exchange; default) vs the reference's RAP (P, local, P^T).
set -eu
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
pr() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], 'MDoF/s', d['ms_per_step'], 'ms/step', d['roofline']['kernel_ms_avg'], 'kernel ms')" "$1" "$2"; }
timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > "$O/dc_n1.json"; pr "$O/dc_n1.json" "N=1"
for dc in overlap rap; do
for rw in ${RANKS:-3:8 0:8 7:8 1:2}; do
  r=${rw%%:*}; n=${rw##*:}
  ECM2_DECOMP=$dc timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --emulate-rank $r --emulate-world $n > "$O/dc_${dc}_${r}_${n}.json"
  pr "$O/dc_${dc}_${r}_${n}.json" "rank $r/$n $dc"
done
done
