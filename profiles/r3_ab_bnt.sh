#!/bin/bash
# Same-box A/Bs (C5): b = HEAD; c = the brick kernel's per-point qdata pairs loaded nontemporal;
# d = the summation pass's partial-slot loads nontemporal.
set -uo pipefail
bash profiles/ab_libs.sh bnt_c5 "libecm2pa_b.so libecm2pa_c.so libecm2pa_d.so" --workload c5 --steps 50 --warmup 5 || exit $?
bash profiles/ab_libs.sh bnt_c4e "libecm2pa_b.so libecm2pa_d.so" --workload c4 --numbering entity --variants 0 --steps 50 --warmup 5 || exit $?
