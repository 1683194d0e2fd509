# round 5, call 31: the driver's bench command three times on one box (run-to-run spread at HEAD)
set -o pipefail
O=gpurun_out/r5/gpu31
mkdir -p $O
for k in 1 2 3; do
  timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_$k.json 2> $O/bench_$k.err || { tail -20 $O/bench_$k.err; exit 1; }
  python3 -c "import json; b=json.loads(open('$O/bench_$k.json').read().strip().splitlines()[-1]); print('run $k', b['value'], b['ms_per_step'], b['roofline']['kernel_ms_avg'], 'drop_in', b['drop_in']['value'], 'entity', b['entity_numbering']['value'], 'pcg', b['pcg_iteration']['iteration_ms'])"
done
