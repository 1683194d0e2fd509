# round 6, call 20: the smooth-state SDIRK33 steps at configs[4] size against the oracle fixtures (converged, fixed 8,
# the shifted state fixed 8)
set -o pipefail
O=gpurun_out/r6/gpu20
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -q -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_configs.py -k "smooth or shifted" > $O/tests_smooth.txt 2>&1; rc=$?
grep "c5 s" $O/tests_smooth.txt; tail -1 $O/tests_smooth.txt; exit $rc
