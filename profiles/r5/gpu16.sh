# round 5, call 16: the ex16p SDIRK33 step on the bench line (C4 default and C5)
set -o pipefail
O=gpurun_out/r5/gpu16
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_bench.py -m gpu \
  > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for wl in c4 c5; do
  timeout -k 10 400 python -u bench.py --workload $wl --steps 20 --warmup 5 --variants 0 --full-layout 0 \
    > $O/bench_$wl.json 2> $O/bench_$wl.err || { tail -20 $O/bench_$wl.err; exit 1; }
  python3 -c "import json; b = json.loads(open('$O/bench_$wl.json').read().strip().splitlines()[-1]); print('$wl', b['value'], b['pcg_iteration']['iteration_ms'], b['sdirk_step'])"
done
