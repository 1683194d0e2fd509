#!/bin/bash
# one box: the nontemporal-load A/Bs (r3_ab_bnt.sh), then collect_r3.sh set a at 1eedce8
set -uo pipefail
bash profiles/r3_ab_bnt.sh || exit $?
COMMIT=1eedce8 bash profiles/collect_r3.sh a || exit $?
