# round 5, call 15: the diagonal kept per assembly -- parity, solver, config and bench tests
set -o pipefail
O=gpurun_out/r5/gpu15
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_solvers.py tests/test_gpu_configs.py tests/test_distributed.py tests/test_examples.py \
  tests/test_bench.py tests/test_gpu_snapshot_laws.py -m gpu > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
