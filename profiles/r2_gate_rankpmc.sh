#!/bin/bash
# HBM bytes of one emulated rank's kernels (member mode) at N = 8 and 4: kernel trace + FETCH + WRITE passes
set -uo pipefail
bash profiles/run_profile.sh c4_n8_member3 --loopback 8 --member 3 --steps 30 --warmup 5 --full-layout 0 || exit $?
bash profiles/run_profile.sh c4_n4_member1 --loopback 4 --member 1 --steps 30 --warmup 5 --full-layout 0 || exit $?
