#!/bin/bash
# GPU suite at the tree (even/odd brick contractions on), then a same-box A/B on C5 (p = 4 brick
# kernel): b = the same tree built with -DECM2_BRICK_EO=0 (plain contractions) vs c = even/odd;
# d, e = c with summation-pass timing probes (wrong results, timing only): d = runs whose dofs are
# not unit-stride store by entry index (contiguous), e = no stores
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r3eo
mkdir -p "$O"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
rc=$?
tail -3 "$O/pytest_gpu.log"; grep -E "FAILED|ERROR" "$O/pytest_gpu.log" | head -20
[ $rc -eq 0 ] || exit $rc
bash profiles/ab_libs.sh eo_c5 "libecm2pa_b.so libecm2pa_c.so libecm2pa_d.so libecm2pa_e.so" --workload c5 --steps 50 --warmup 5 || exit $?
