# round 5, third GPU call: the snapshot tests (all laws, p = 2 and bricks), the parity files, then the C5 A/B
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 1000 python -u -m pytest --maxfail=5 -q --timeout 300 --timeout-method thread --durations=15 \
  tests/test_gpu_snapshot_laws.py tests/test_gpu_timed_forms.py tests/test_gpu_parity.py tests/test_gpu_configs.py \
  > gpurun_out/r5/tests3.txt 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r5/tests3.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 bash profiles/r5/ab_c5.sh > gpurun_out/r5/ab_c5.txt 2>&1
