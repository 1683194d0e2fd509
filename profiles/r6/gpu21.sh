# round 6, call 21: the operator side of the smooth-state SDIRK gap (profiles/r6/sdirk_gap_probe.py) at configs[4] size
set -o pipefail
O=gpurun_out/r6/gpu21
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u profiles/r6/sdirk_gap_probe.py > $O/probe.txt 2>&1; rc=$?
cat $O/probe.txt; exit $rc
