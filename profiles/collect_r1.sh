#!/bin/bash
# Round-1 evidence on one MI355X: kernel-trace + PMC profiles of C2 / C3 / C4 / C5 (reduced by
# profiles/pmc_reduce.py), then the default bench line (C2, with its CPU baseline), the C3 /
# C4 / C5 lines, and the partitioned path (loopback) for C4.
set -euo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$O"
bash profiles/run_profile.sh c2 --steps 50 --warmup 5 > "$O/prof_c2.log" 2>&1
bash profiles/run_profile.sh c3 --workload c3 --steps 20 --warmup 3 > "$O/prof_c3.log" 2>&1
bash profiles/run_profile.sh c4 --workload c4 --steps 20 --warmup 3 > "$O/prof_c4.log" 2>&1
bash profiles/run_profile.sh c5 --workload c5 --steps 20 --warmup 3 > "$O/prof_c5.log" 2>&1
# pin each dominant kernel's PMC bytes as bench.py's roofline.traffic source (copied to profiles/)
mkdir -p "$O/pins"
for w in c2 c3 c4 c5; do
  lay=$(python3 -c "import json; print(json.loads(open('$O/prof_$w/bench_trace.json').read().strip().splitlines()[-1])['config']['qdata_layout'])")
  key=apply; [ "$w" = c5 ] && key=apply_brick
  python3 profiles/pmc_pin.py "$O/prof_$w" "$w" "$key" > "$O/pins/pmc_${w}_n1_${lay}.json"
done
timeout -k 10 300 python3 bench.py > "$O/bench_c2.json" 2> "$O/bench_c2.err"
timeout -k 10 300 python3 bench.py --workload c3 --steps 30 --warmup 5 --no-cpu-baseline > "$O/bench_c3.json" 2> "$O/bench_c3.err"
timeout -k 10 300 python3 bench.py --workload c4 --steps 50 --warmup 5 > "$O/bench_c4.json" 2> "$O/bench_c4.err"
timeout -k 10 300 python3 bench.py --workload c5 --steps 30 --warmup 5 > "$O/bench_c5.json" 2> "$O/bench_c5.err"
timeout -k 10 300 python3 bench.py --workload c4 --steps 50 --warmup 5 --loopback 8 --no-cpu-baseline > "$O/bench_c4_lb8.json" 2> "$O/bench_c4_lb8.err"
cat "$O"/bench_*.json
