# round 6, call 22: VERDICT r5 item 3 -- brick partial slots with every face group on its own 128-B lines
# (-DECM2_BRICK_SLOT_ALIGN=16, libecm2pa_al.so): parity on the brick forms, then the C5 Mult and its summation
# pass against the default build on the same box
set -o pipefail
O=gpurun_out/r6/gpu22
mkdir -p $O
export TMPDIR=/tmp
L=cardiac-ablation-ecm2_amd/lib
timeout -k 10 600 python3 -u profiles/pytest_lib.py $L/libecm2pa_al.so -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_configs.py tests/test_gpu_timed_forms.py tests/test_gpu_parity.py -k "c5 or p4 or brick or line or order4 or high" \
  > $O/tests_al.txt 2>&1 || { tail -40 $O/tests_al.txt; exit 1; }
tail -1 $O/tests_al.txt
A="--workload c5 --variants 0 --full-layout 0 --sdirk 0 --pcg-iters 0 --no-cpu-baseline --steps 40 --warmup 5"
for rep in 1 2; do
  for v in libecm2pa.so libecm2pa_al.so; do
    timeout -k 10 300 python3 profiles/ab_lib.py $L/$v $A > $O/c5_${v}_$rep.json 2> $O/c5_${v}_$rep.err || exit 1
    python3 -c "import json; d=json.loads(open('$O/c5_${v}_$rep.json').read().strip().splitlines()[-1]); print('$v rep $rep', d['value'], 'MDoF/s', d['ms_per_step'], 'ms kernel', d['roofline']['kernel_ms_avg'])"
  done
done
for v in libecm2pa.so libecm2pa_al.so; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- python3 profiles/ab_lib.py $L/$v $A > $O/prof_$v.log 2>&1 || exit 1
  f=$(find $O/prof_$v -name '*kernel_stats.csv' | head -1)
  python3 - "$f" "$v" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    n = r["Name"]
    if "k_sum_partials" in n or "k_apply_brick" in n:
        print(sys.argv[2], n.split("(")[0][-60:], r["Calls"], "avg us", round(float(r["AverageNs"]) / 1e3, 2))
PY
done
