# round 5, call 10: the one-pass dot and the stopping test fused into the PCG step -- PCG / solver /
# distributed GPU tests, then the member emulation's marginal PCG iteration at N = 1 and 8
set -o pipefail
O=gpurun_out/r5/gpu10
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_solvers.py tests/test_distributed.py tests/test_gpu_configs.py tests/test_examples.py \
  tests/test_bench.py -m gpu > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
EXTRA="--pcg-iters 50 --variants 0" timeout -k 10 600 bash profiles/member_emul.sh 2 4 8 > $O/member_emul.txt 2>&1 || { cat $O/member_emul.txt; exit 1; }
cat $O/member_emul.txt
