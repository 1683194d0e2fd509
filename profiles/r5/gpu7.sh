# round 5, call 7: curved-mesh / snapshot-law / timed-C5 GPU tests at HEAD, then the summation-pass A/B
# (ECM2_SUM_EPT = plan entries per thread: 1 = 256-thread workgroups, 2 = 128, 4 = 64; same LDS
# staging), two interleaved repetitions on C4, C4 entity numbering, C3 and C5, then the member emulation.
set -o pipefail
O=gpurun_out/r5/gpu7
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_parity.py::test_curved_mesh_jacobians tests/test_gpu_snapshot_laws.py \
  tests/test_gpu_timed_forms.py::test_timed_c5_form > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -3 $O/tests.txt
for ept in 2 4; do  # the narrower summation workgroups against the oracle before timing them
  ECM2_SUM_EPT=$ept timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_parity.py > $O/parity_e$ept.txt 2>&1 || { tail -30 $O/parity_e$ept.txt; exit 1; }
  tail -1 $O/parity_e$ept.txt
done
run() {  # tag ept bench-args
  local tag=$1 ept=$2; shift 2
  ECM2_SUM_EPT=$ept timeout -k 10 300 python -u bench.py "$@" --full-layout 0 --variants 0 --no-cpu-baseline \
    > $O/$tag.json 2> $O/$tag.err || return 1
  python3 -c "import json,sys; b=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=b['roofline']; print(sys.argv[2], b['value'], 'MDoF/s', b['ms_per_step'], 'ms/Mult', 'kernel', r['kernel_ms_avg'], 'rest', round(b['ms_per_step'] - r['kernel_ms_avg'], 5))" $O/$tag.json $tag
}
for rep in 1 2; do
  for ept in 1 2 4; do
    run c4_e${ept}_$rep $ept --workload c4 --steps 50 --warmup 5 &&
    run c4ent_e${ept}_$rep $ept --workload c4 --numbering entity --steps 50 --warmup 5 &&
    run c5_e${ept}_$rep $ept --workload c5 --steps 30 --warmup 5 &&
    run c3_e${ept}_$rep $ept --workload c3 --steps 30 --warmup 5 || exit 1
  done
done
