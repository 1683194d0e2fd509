# round 6, call 4: PCG vector kernels with 16-byte accesses and a 1,024-thread final dot pass -- parity
# (the PCG / SDIRK tests), the marginal PCG iteration A/B against the previous build (libecm2pa_r6a.so,
# HEAD 73d3525), and the HBM copy probe (profiles/calib/copy_probe.hip)
set -o pipefail
O=gpurun_out/r6/gpu4
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_solvers.py tests/test_distributed.py -k "pcg or PCG or ode or sdirk or member" > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
timeout -k 10 120 profiles/calib/copy_probe > $O/copy_probe.json || exit 1
cat $O/copy_probe.json
A="--variants 0 --full-layout 0 --sdirk 0 --no-cpu-baseline --steps 30 --warmup 5 --pcg-iters 20"
for rep in 1 2; do
  for v in libecm2pa_r6a.so libecm2pa.so; do
    for w in c4 c5; do
      timeout -k 10 300 python3 profiles/ab_lib.py cardiac-ablation-ecm2_amd/lib/$v $A --workload $w > $O/pcg_${v}_${w}_$rep.json 2> $O/pcg_${v}_${w}_$rep.err || exit 1
      python3 -c "import json; d=json.loads(open('$O/pcg_${v}_${w}_$rep.json').read().strip().splitlines()[-1]); print('$v $w rep $rep', d['value'], d['ms_per_step'], 'pcg_it_ms', d['pcg_iteration']['iteration_ms'])"
    done
  done
done
