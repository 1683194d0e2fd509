# round 6, call 27: C4 N = 8 member emulation repeated twice (gpu26's member 0 read 0.090 ms against 0.061-0.066 in every earlier run)
set -o pipefail
O=gpurun_out/r6/gpu27
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  TAG=_final27_$rep EXTRA='--pcg-iters 50 --variants 0 --sdirk 0' bash profiles/member_emul.sh 8 > $O/member_c4_$rep.txt 2>&1 || { tail -5 $O/member_c4_$rep.txt; exit 1; }
  cat $O/member_c4_$rep.txt
done
