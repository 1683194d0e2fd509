# round-6 gate at HEAD: the whole GPU suite (as the driver runs it), smoke(), the default bench line (the driver's
# command) twice, and a kernel trace (rocprofv3 --kernel-trace --stats) of the default line -- gpurun_out/r6/gate/
set -o pipefail
O=${O:-gpurun_out/r6/gate}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=15 \
  > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
tail -2 $O/smoke.txt
for k in 1 2; do
  timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_$k.json 2> $O/bench_$k.err || { tail -20 $O/bench_$k.err; exit 1; }
  python3 -c "
import json; b = json.loads(open('$O/bench_$k.json').read().strip().splitlines()[-1])
print('run $k value', b['value'], 'ms', b['ms_per_step'], 'kernel', b['roofline']['kernel_ms_avg'], 'frac', b['roofline']['frac'], 'fp64', b['roofline']['fp64']['frac'], 'copy', b['roofline']['stream_copy_gbs'], 'pcg', b['pcg_iteration']['iteration_ms'], 'sdirk', b['sdirk_step']['step_ms'])
for k in ('entity_numbering', 'trilinear', 'drop_in', 'full_layout', 'pennes', 'ex16'):
    print('   ', k, b[k]['value'], b[k]['ms_per_step'])
print('    cpu', b['cpu_baseline']['value'], b['cpu_baseline']['cores'])
"
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/prof_bench.json 2> $O/prof_bench.err || { tail -20 $O/prof_bench.err; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp $f $O/kernel_stats.csv
head -12 $O/kernel_stats.csv | cut -c1-160
