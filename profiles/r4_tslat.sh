#!/bin/bash
# Round 4: the k(T) snapshot in the lattice-map blocks' slot order (the reference's numbering) --
# parity, then same-box A/B against the dof-ordered snapshot (tsdof) on C4 with the reference's
# numbering and, as a control, the structured numbering.
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r4tslat
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "coefficient_snapshot or full_size_c4 or attribute_markers" > "$O/tests.txt" 2>&1 || { tail -40 "$O/tests.txt"; exit 1; }
tail -1 "$O/tests.txt"
bash profiles/ab_libs.sh tslat_ent "libecm2pa.so libecm2pa_tsdof.so" --workload c4 --numbering entity --steps 30 --warmup 5 --variants 0 || exit $?
bash profiles/ab_libs.sh tslat_str "libecm2pa.so libecm2pa_tsdof.so" --workload c4 --steps 30 --warmup 5 --variants 0 || exit $?
