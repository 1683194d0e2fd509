# round 6, call 15: CGSolver's den folded into the p >= 3 brick kernel at its end (x line gathered again) -- parity (the energy tests, the brick /
# line kernels, configs[4] at size), then the C5 Mult and PCG iteration A/B against f718aa1 (libecm2pa_r6b.so)
set -o pipefail
O=gpurun_out/r6/gpu15
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_configs.py -k "energy or brick or line or pcg or c5" > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
A="--variants 0 --full-layout 0 --sdirk 0 --no-cpu-baseline --steps 30 --warmup 5 --pcg-iters 20"
for rep in 1 2 3; do
  for v in libecm2pa_r6b.so libecm2pa.so; do
    for w in c5 c4; do
      timeout -k 10 300 python3 profiles/ab_lib.py cardiac-ablation-ecm2_amd/lib/$v $A --workload $w > $O/pcg_${v}_${w}_$rep.json 2> $O/pcg_${v}_${w}_$rep.err || exit 1
      python3 -c "import json; d=json.loads(open('$O/pcg_${v}_${w}_$rep.json').read().strip().splitlines()[-1]); print('$v $w rep $rep', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_avg'], 'pcg_it_ms', d['pcg_iteration']['iteration_ms'])"
    done
  done
done
