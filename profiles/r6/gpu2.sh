# round 6, call 2: the GPU suite at the PCG restructure + padded LDS; the marginal PCG iteration
# A/B (round-5 build vs HEAD) on C4 and C5, same box
set -o pipefail
O=gpurun_out/r6/gpu2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -3 $O/tests.txt
A="--variants 0 --full-layout 0 --sdirk 0 --no-cpu-baseline --steps 30 --warmup 5 --pcg-iters 20"
for rep in 1 2; do
  for v in libecm2pa_r5base.so libecm2pa.so libecm2pa_en.so; do
    for w in c4 c5; do
      timeout -k 10 300 python3 profiles/ab_lib.py cardiac-ablation-ecm2_amd/lib/$v $A --workload $w > $O/pcg_${v}_${w}_$rep.json 2> $O/pcg_${v}_${w}_$rep.err || exit 1
      python3 -c "import json; d=json.loads(open('$O/pcg_${v}_${w}_$rep.json').read().strip().splitlines()[-1]); print('$v $w rep $rep', d['value'], d['ms_per_step'], 'pcg_it_ms', d['pcg_iteration']['iteration_ms'])"
    done
  done
done
