#!/bin/bash
# Emulated ranks of the weak-scaled C2 partition (bench.py --emulate-rank/--emulate-world: one
# rank alone, exchanges = local copies) against the single-GPU C2 line, with and without the
# CU-masked comm stream (ECM2_COMM_CUS = 16 / 0).
set -eu
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
pr() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], d['value'], 'MDoF/s', d['ms_per_step'], 'ms/step', r['kernel_ms_avg'], 'kernel ms')" "$1" "$2"; }
timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > "$O/emu_n1.json"; pr "$O/emu_n1.json" "N=1"
for cus in ${CUS:-16 0}; do
for rw in ${RANKS:-1:2 3:8 0:8}; do
  r=${rw%%:*}; n=${rw##*:}
  ECM2_COMM_CUS=$cus timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --emulate-rank $r --emulate-world $n > "$O/emu_${r}_${n}_${cus}.json"
  pr "$O/emu_${r}_${n}_${cus}.json" "rank $r/$n comm_cus=$cus"
done
done
