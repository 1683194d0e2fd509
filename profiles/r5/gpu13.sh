# round 5, call 13: two-pass dots with the stopping test in the final pass, the host polling the
# mirror's progress mark (no per-iteration events) -- solver tests, then the member emulation's PCG iteration
set -o pipefail
O=gpurun_out/r5/gpu13
mkdir -p $O
timeout -k 10 120 ./profiles/calib/dot_probe > $O/dot_probe.txt 2>&1 || { cat $O/dot_probe.txt; exit 1; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_solvers.py tests/test_distributed.py tests/test_gpu_configs.py tests/test_examples.py \
  tests/test_bench.py -m gpu > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
EXTRA="--pcg-iters 50 --variants 0" timeout -k 10 600 bash profiles/member_emul.sh 2 4 8 > $O/member_emul.txt 2>&1 || { cat $O/member_emul.txt; exit 1; }
cat $O/member_emul.txt
