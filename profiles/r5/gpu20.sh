# round 5, call 20: the summation pass with each entry's run index loaded (ECM2_SUM_RIX=1) instead of
# the binary search over the block's runs in LDS -- parity with it on (and the solver tests at HEAD),
# then two interleaved repetitions on C4, C4 entity numbering, C3 and C5
set -o pipefail
O=gpurun_out/r5/gpu20
mkdir -p $O
ECM2_SUM_RIX=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_solvers.py tests/test_gpu_timed_forms.py > $O/parity_rix.txt 2>&1 || { tail -30 $O/parity_rix.txt; exit 1; }
tail -1 $O/parity_rix.txt
X="--variants 0 --full-layout 0 --no-cpu-baseline --sdirk 0 --pcg-iters 0"
run() {  # tag rix bench-args
  local tag=$1 rix=$2; shift 2
  ECM2_SUM_RIX=$rix timeout -k 10 300 python -u bench.py "$@" $X > $O/$tag.json 2> $O/$tag.err || return 1
  python3 -c "import json,sys; b=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=b['roofline']; print(sys.argv[2], b['value'], 'MDoF/s', b['ms_per_step'], 'ms/Mult', 'kernel', r['kernel_ms_avg'], 'rest', round(b['ms_per_step'] - r['kernel_ms_avg'], 5))" $O/$tag.json $tag
}
for rep in 1 2; do
  for rix in 0 1; do
    run c4_r${rix}_$rep $rix --workload c4 --steps 50 --warmup 5 &&
    run c4ent_r${rix}_$rep $rix --workload c4 --numbering entity --steps 50 --warmup 5 &&
    run c5_r${rix}_$rep $rix --workload c5 --steps 30 --warmup 5 &&
    run c3_r${rix}_$rep $rix --workload c3 --steps 30 --warmup 5 || exit 1
  done
done
