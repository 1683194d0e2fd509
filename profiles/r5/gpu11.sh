# round 5, call 11: kernel trace of one N = 8 member's PCG iterations (what a rank's iteration is made of)
set -o pipefail
O=gpurun_out/r5/gpu11
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $O/trace -o run --output-format csv \
  -- python3 bench.py --workload c4 --loopback 8 --member 3 --steps 20 --warmup 3 --no-cpu-baseline --pcg-iters 50 \
  > $O/bench.json 2> $O/trace.err || { tail -20 $O/trace.err; exit 1; }
tail -1 $O/bench.json | cut -c1-400
