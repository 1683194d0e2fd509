# round 5, second GPU call: the generalised snapshot, the SDIRK step at size, the full parity files, one bench
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 900 python -u -m pytest --maxfail=3 -q --timeout 300 --timeout-method thread --durations=15 \
  tests/test_gpu_snapshot_laws.py tests/test_gpu_parity.py tests/test_gpu_timed_forms.py \
  "tests/test_gpu_configs.py::test_c5_sdirk_step_full_size" \
  tests/test_distributed.py -k "not nothing" -m gpu > gpurun_out/r5/tests2.txt 2>&1 &&
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --full-layout 0 > gpurun_out/r5/bench2.json 2> gpurun_out/r5/bench2.err
