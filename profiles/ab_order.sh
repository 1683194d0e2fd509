#!/bin/bash
# Emulated middle rank (3 of 8) of the weak-scaled C2 partition: enqueue order (interior first
# or after the exchange chain) x graph capture x the runtime's graph packet capture.
set -eu
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
pr() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], 'MDoF/s', d['ms_per_step'], 'ms/step')" "$1" "$2"; }
timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > "$O/or_n1.json"; pr "$O/or_n1.json" "N=1"
for first in 1 0; do
for g in 1 0; do
  ECM2_INTERIOR_FIRST=$first ECM2_PAR_GRAPH=$g timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --emulate-rank 3 --emulate-world 8 > "$O/or_${first}_${g}.json"
  pr "$O/or_${first}_${g}.json" "rank 3/8 interior_first=$first graph=$g"
done
done
for pc in 0 1; do
  DEBUG_CLR_GRAPH_PACKET_CAPTURE=$pc ECM2_INTERIOR_FIRST=1 ECM2_PAR_GRAPH=1 timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --emulate-rank 3 --emulate-world 8 > "$O/or_pc$pc.json"
  pr "$O/or_pc$pc.json" "rank 3/8 interior_first=1 graph=1 packet_capture=$pc"
done
