#!/bin/bash
# Round-3 close: the emulated per-rank Mult with the interleaved-pass member mode (median of 3 passes per
# member), OVERLAP and RAP slabs, N = 2 / 4 / 8, and N = 1 on the same box.
set -uo pipefail
bash profiles/member_emul.sh 2 4 8 || exit $?
ECM2_DECOMP=rap TAG=_rap bash profiles/member_emul.sh 8 || exit $?
