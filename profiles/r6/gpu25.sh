# round 6, call 25: the diagonal flux in the stored-pair AFFINE kernel too (k_apply_tpe_sf<..., CD>, what a
# z-slab rank runs) -- parity (timed forms, partitioned groups and members), then C4 N = 8 member emulation
# against ECM2_CDIAG=0 on the same box
set -o pipefail
O=gpurun_out/r6/gpu25
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_timed_forms.py \
  tests/test_distributed.py tests/test_gpu_configs.py -k "diagonal or snapshot or loopback or member or slabs or boxes or lattice_addressing or timed" \
  > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for rep in 1 2; do
  for c in 1 0; do
    ECM2_CDIAG=$c TAG=_cd${c}_$rep EXTRA='--pcg-iters 50 --variants 0 --sdirk 0' bash profiles/member_emul.sh 8 > $O/member_cd${c}_$rep.txt 2>&1 || { tail -5 $O/member_cd${c}_$rep.txt; exit 1; }
    echo "cdiag=$c rep $rep"; cat $O/member_cd${c}_$rep.txt
  done
done
