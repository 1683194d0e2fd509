#!/bin/bash
# Round-3 close at HEAD: GPU suite + the default bench line (r3_gate_head.sh), then one SQ-counter pass
# each on C5, C4 and C4 with the reference's numbering (where the apply kernels' wave cycles go).
set -uo pipefail
bash profiles/r3_gate_head.sh || exit $?
bash profiles/sq_pass.sh r3_c5 --workload c5 --steps 20 --warmup 3 --full-layout 0 > /dev/null || exit $?
bash profiles/sq_pass.sh r3_c4 --workload c4 --steps 20 --warmup 3 --full-layout 0 --variants 0 > /dev/null || exit $?
bash profiles/sq_pass.sh r3_c4ent --workload c4 --numbering entity --steps 20 --warmup 3 --full-layout 0 --variants 0 > /dev/null || exit $?
echo sq done
