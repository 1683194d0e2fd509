# round 5, fourth GPU call: the q1d = p + 3 and snapshot tests, then the C5 A/B (grid pass K, brick snapshot)
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 600 python -u -m pytest --maxfail=5 -q --timeout 300 --timeout-method thread \
  tests/test_gpu_snapshot_laws.py "tests/test_gpu_parity.py::test_integration_rule_q1d" tests/test_gpu_timed_forms.py \
  "tests/test_gpu_configs.py::test_c5_full_size" "tests/test_gpu_configs.py::test_c5_p4_cartesian_32" \
  "tests/test_gpu_configs.py::test_lattice_addressing_matches_map_path" \
  > gpurun_out/r5/tests4.txt 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r5/tests4.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 bash profiles/r5/ab_c5b.sh > gpurun_out/r5/ab_c5b.txt 2>&1
