#!/bin/bash
# Round-1 evidence on one MI355X: profile of the default bench (C2), the default bench
# line with its CPU baseline, C4 on one GPU, and the partitioned path (loopback) for C4.
set -euo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$O"
bash profiles/run_profile.sh c2 > "$O/prof_c2.log" 2>&1
timeout -k 10 300 python3 bench.py > "$O/bench_c2.json" 2> "$O/bench_c2.err"
timeout -k 10 300 python3 bench.py --workload c4 --steps 50 --warmup 5 > "$O/bench_c4.json" 2> "$O/bench_c4.err"
timeout -k 10 300 python3 bench.py --workload c4 --steps 50 --warmup 5 --loopback 8 --no-cpu-baseline > "$O/bench_c4_lb8.json" 2> "$O/bench_c4_lb8.err"
timeout -k 10 300 python3 bench.py --loopback 2 --steps 100 --no-cpu-baseline > "$O/bench_c2_lb2.json" 2> "$O/bench_c2_lb2.err"
cat "$O"/bench_*.json
