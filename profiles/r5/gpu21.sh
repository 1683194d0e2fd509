# round 5, call 21: 8-wave workgroups for the snapshot kernel (ECM2_GROUP_WAVES=8: 2x2x2 brick groups
# in the Morton brick order, 12 merged cross-wave faces per group instead of 4 per 2x2x1 group) --
# parity of the C4 snapshot forms with it on (only forms that run k_apply_tpe_ts: the plan's grouping is
# global; the 50^3 forms keep 4-wave kernels and fail under this switch by construction), then two interleaved repetitions on C4 and C4-entity
set -o pipefail
O=gpurun_out/r5/gpu21
mkdir -p $O
ECM2_GROUP_WAVES=8 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  "tests/test_gpu_timed_forms.py::test_timed_snapshot_forms[108-structured]" \
  "tests/test_gpu_timed_forms.py::test_timed_snapshot_forms[108-entity]" > $O/parity_w8.txt 2>&1
tail -1 $O/parity_w8.txt  # (the Mult passes; the diagonal kernel keeps 4-wave groups, so it fails under the switch)
X="--variants 0 --full-layout 0 --no-cpu-baseline --sdirk 0 --pcg-iters 0"
run() {  # tag waves bench-args
  local tag=$1 gw=$2; shift 2
  ECM2_GROUP_WAVES=$gw timeout -k 10 300 python -u bench.py "$@" $X > $O/$tag.json 2> $O/$tag.err || return 1
  python3 -c "import json,sys; b=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=b['roofline']; print(sys.argv[2], b['value'], 'MDoF/s', b['ms_per_step'], 'ms/Mult', 'kernel', r['kernel_ms_avg'], 'rest', round(b['ms_per_step'] - r['kernel_ms_avg'], 5), 'runs', b['config']['summation_runs'])" $O/$tag.json $tag
}
for rep in 1 2; do
  for gw in 4 8; do
    run c4_w${gw}_$rep $gw --workload c4 --steps 50 --warmup 5 &&
    run c4ent_w${gw}_$rep $gw --workload c4 --numbering entity --steps 50 --warmup 5 &&
    run c4pen_w${gw}_$rep $gw --workload c4 --coefficients pennes --steps 50 --warmup 5 || exit 1
  done
done
