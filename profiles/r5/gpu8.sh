# round 5, call 8: the member operator (one rank's PCG iteration) tests, then the member emulation at
# HEAD with the PCG iteration beside the Mult (profiles/r5_member_emul.txt)
set -o pipefail
O=gpurun_out/r5/gpu8
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_distributed.py::test_gpu_member_operator_pcg tests/test_bench.py::test_bench_loopback_group_and_member_lines \
  > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -3 $O/tests.txt
EXTRA="--pcg-iters 50" timeout -k 10 900 bash profiles/member_emul.sh 2 4 8 > $O/member_emul.txt 2>&1 || { cat $O/member_emul.txt; exit 1; }
cat $O/member_emul.txt
