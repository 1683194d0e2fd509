# round-5 gate at HEAD: the whole GPU suite (as the driver runs it), smoke(), then the default bench
# line (the driver's command) -- results under gpurun_out/r5/gate/
set -o pipefail
O=gpurun_out/r5/gate
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=15 \
  > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
tail -2 $O/smoke.txt
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; b = json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('value', b['value'], 'ms', b['ms_per_step'], 'frac', b['roofline']['frac'], 'pcg', b.get('pcg_iteration'))
for k in ('entity_numbering', 'trilinear', 'drop_in', 'full_layout', 'pennes', 'ex16'):
    print(k, b[k]['value'], b[k]['ms_per_step'])
"
