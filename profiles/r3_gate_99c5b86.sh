#!/bin/bash
# GPU suite at 99c5b86 (nontemporal brick qdata), C5/C3 evidence (collect_r3.sh set b), then a same-box
# A/B: e = the brick kernel's partial-slot stores nontemporal, against b = the tree.
set -uo pipefail
COMMIT=99c5b86 bash profiles/collect_r3.sh b t || exit $?
bash profiles/ab_libs.sh pnt_c5 "libecm2pa_b.so libecm2pa_e.so" --workload c5 --steps 50 --warmup 5 || exit $?
