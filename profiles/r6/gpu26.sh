# round 6, call 26: member emulation at the final tree (C4 N = 2 / 4 / 8, C5 N = 8), as profiles/r6/gpu10.sh
set -o pipefail
O=gpurun_out/r6/gpu26
mkdir -p $O
export TMPDIR=/tmp
TAG=_final EXTRA='--pcg-iters 50 --variants 0 --sdirk 0' bash profiles/member_emul.sh 2 4 8 > $O/member_c4.txt 2>&1 || { tail -5 $O/member_c4.txt; exit 1; }
cat $O/member_c4.txt
WL=c5 TAG=_final EXTRA='--pcg-iters 20 --variants 0 --sdirk 0' bash profiles/member_emul.sh 8 > $O/member_c5.txt 2>&1 || { tail -5 $O/member_c5.txt; exit 1; }
cat $O/member_c5.txt
