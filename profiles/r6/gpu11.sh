# round 6, call 11: the gather dealt per 64-slot step for the write banks (LatticeTsGather) -- parity, A/B against f718aa1,
# SQ counters
set -o pipefail
O=gpurun_out/r6/gpu11
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_timed_forms.py tests/test_gpu_snapshot_laws.py tests/test_gpu_parity.py -k "snapshot or timed or energy or laws or Timed" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -3 $O/tests.txt
A="--variants 0 --full-layout 0 --sdirk 0 --pcg-iters 0 --no-cpu-baseline --steps 50 --warmup 5"
for rep in 1 2; do
  for v in libecm2pa_r6b.so libecm2pa.so; do
    for num in structured entity; do
      timeout -k 10 300 python3 profiles/ab_lib.py cardiac-ablation-ecm2_amd/lib/$v $A --numbering $num > $O/ab_${v}_${num}_$rep.json 2> $O/ab_${v}_${num}_$rep.err || exit 1
      python3 -c "import json; d=json.loads(open('$O/ab_${v}_${num}_$rep.json').read().strip().splitlines()[-1]); print('$v $num rep $rep', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_avg'])"
    done
  done
done
SQ_ARGS="--workload c4 --steps 20 --warmup 3 --variants 0 --full-layout 0 --sdirk 0 --pcg-iters 0"
bash profiles/sq_pass.sh r6_c4_tsg $SQ_ARGS > /dev/null && cp gpurun_out/sq_r6_c4_tsg/sq_summary.json $O/sq_c4_tsg.json && python3 -c "
import json; d=json.load(open('$O/sq_c4_tsg.json'))
for k,v in d.items():
    if 'tpe_ts' in k or 'sum_partials' in k: print(k[:60], {kk: v[kk] for kk in v if 'LDS' in kk or 'WAIT_ANY' in kk or 'VALU' in kk})
"
