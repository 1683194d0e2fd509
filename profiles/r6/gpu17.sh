# round 6, call 17: the smooth-state converged SDIRK33 step at configs[4] size against the oracle's fixture
set -o pipefail
O=gpurun_out/r6/gpu17
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -s --timeout 500 --timeout-method thread -m gpu tests/test_gpu_configs.py -k "smooth_converged or sdirk_step_full_size" > $O/tests.txt 2>&1
rc=$?
grep -E "relerr|passed|failed|Error" $O/tests.txt | tail -8
exit $rc
