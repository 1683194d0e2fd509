# round 6, call 10: PCG with the grid-stride 16-byte step, flat chunked dots, 1,024-thread final pass, flat STREAM copy --
# PCG / SDIRK parity, the PCG iteration A/B against libecm2pa_r6a.so (73d3525), member emulation (C4 N = 2/4/8,
# C5 N = 8) at this tree
set -o pipefail
O=gpurun_out/r6/gpu10
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_solvers.py tests/test_distributed.py tests/test_gpu_configs.py -k "pcg or PCG or ode or sdirk or member" > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
A="--variants 0 --full-layout 0 --sdirk 0 --no-cpu-baseline --steps 30 --warmup 5 --pcg-iters 20"
for rep in 1 2; do
  for v in libecm2pa_r6a.so libecm2pa.so; do
    for w in c4 c5; do
      timeout -k 10 300 python3 profiles/ab_lib.py cardiac-ablation-ecm2_amd/lib/$v $A --workload $w > $O/pcg_${v}_${w}_$rep.json 2> $O/pcg_${v}_${w}_$rep.err || exit 1
      python3 -c "import json; d=json.loads(open('$O/pcg_${v}_${w}_$rep.json').read().strip().splitlines()[-1]); print('$v $w rep $rep', d['value'], d['ms_per_step'], 'pcg_it_ms', d['pcg_iteration']['iteration_ms'], 'copy', d['roofline']['stream_copy_gbs'])"
    done
  done
done
EXTRA='--pcg-iters 50 --variants 0' bash profiles/member_emul.sh 2 4 8 > $O/member_c4.txt 2>&1 || { tail -5 $O/member_c4.txt; exit 1; }
cat $O/member_c4.txt
WL=c5 EXTRA='--pcg-iters 20 --variants 0 --sdirk 0' bash profiles/member_emul.sh 8 > $O/member_c5.txt 2>&1 || { tail -5 $O/member_c5.txt; exit 1; }
cat $O/member_c5.txt
