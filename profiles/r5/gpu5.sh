# round 5, fifth GPU call: the whole GPU suite (as the driver runs it), then the default bench line
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --durations=20 \
  > gpurun_out/r5/tests5.txt 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r5/tests5.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py > gpurun_out/r5/bench5.json 2> gpurun_out/r5/bench5.err
