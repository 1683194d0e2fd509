# round 6, call 19: VERDICT r5 item 1b -- the three-waves-per-SIMD build of k_apply_tpe_sf (libecm2pa_w3.so, second form: no plane sums, one row buffer,
# -DECM2_SF_W3=1): its parity on the partitioned-form tests, then member emulation (C4 N = 8) against the
# default build on the same box
set -o pipefail
O=gpurun_out/r6/gpu19
mkdir -p $O
export TMPDIR=/tmp
L=cardiac-ablation-ecm2_amd/lib
timeout -k 10 600 python3 -u profiles/pytest_lib.py $L/libecm2pa_w3.so -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_distributed.py tests/test_gpu_configs.py -k "loopback or member or slabs or boxes or lattice_addressing" \
  > $O/tests_w3.txt 2>&1 || { tail -40 $O/tests_w3.txt; exit 1; }
tail -2 $O/tests_w3.txt
for rep in 1 2; do
  for v in libecm2pa.so libecm2pa_w3.so; do
    LIB=$L/$v TAG=_${v}_$rep EXTRA='--pcg-iters 50 --variants 0 --sdirk 0' bash profiles/member_emul.sh 8 > $O/member_${v}_$rep.txt 2>&1 || { tail -5 $O/member_${v}_$rep.txt; exit 1; }
    echo "$v rep $rep"; cat $O/member_${v}_$rep.txt
  done
done
timeout -k 10 600 python3 -u -m pytest -x -q -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_configs.py -k "smooth" > $O/tests_smooth.txt 2>&1 || { tail -40 $O/tests_smooth.txt; exit 1; }
grep "c5 smooth" $O/tests_smooth.txt; tail -1 $O/tests_smooth.txt
