# round 5, call 9: the device-driven PCG loop -- full GPU suite, the member emulation's PCG iteration,
# and a kernel trace of 50 PCG iterations on one GPU (the vector kernels' times beside the Mult's)
set -o pipefail
O=gpurun_out/r5/gpu9
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
EXTRA="--pcg-iters 50 --variants 0" timeout -k 10 600 bash profiles/member_emul.sh 8 > $O/member_emul.txt 2>&1 || { cat $O/member_emul.txt; exit 1; }
cat $O/member_emul.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $O/pcgtrace -o run --output-format csv \
  -- python3 bench.py --workload c4 --steps 20 --warmup 3 --variants 0 --full-layout 0 --no-cpu-baseline --pcg-iters 50 \
  > $O/pcg_trace_bench.json 2> $O/pcg_trace.err || { tail -20 $O/pcg_trace.err; exit 1; }
python3 - $O/pcgtrace <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
for row in csv.DictReader(open(f)):
    print(f"{row['Name'][:70]:70s} calls {row['Calls']:>6s} avg_us {float(row['AverageNs'])/1e3:9.2f} total_ms {float(row['TotalDurationNs'])/1e6:9.2f}")
PY
