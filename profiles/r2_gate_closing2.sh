#!/bin/bash
# schedule A/B (reproducible script) + per-rank PMC at N = 2
set -uo pipefail
bash profiles/r2_sched_ab.sh 2 4 8 || exit $?
bash profiles/run_profile.sh c4_n2_member1 --loopback 2 --member 1 --steps 30 --warmup 5 --full-layout 0 > /dev/null || exit $?
