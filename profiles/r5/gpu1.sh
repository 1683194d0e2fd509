# round 5, first GPU call: snapshot probe on partitioned forms, the new parity tests
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 180 python -u profiles/r5/probe_snap_parts.py > gpurun_out/r5/probe_snap_parts.txt 2>&1 &&
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread --durations=0 \
  tests/test_gpu_timed_forms.py tests/test_gpu_configs.py tests/test_gpu_parity.py \
  -k "integration_rule or marker_diagonal or coefficient_snapshot or attribute_markers or timed or sdirk_step_full" \
  > gpurun_out/r5/tests1.txt 2>&1
