#!/bin/bash
# Round 3: the serial PCG loop's fused kernels (pcg_step reducing d.Ad's partials itself; update_d
# with the ConstrainedOperator's ess save; ess restore with the d.Ad partials) -- b = before, c = after.
# Solver tests at c first.  C3 Jacobi-PCG rate (bench.py --workload c3 'pcg'), two reps each.
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/pcgfuse
mkdir -p "$O"
timeout -k 10 600 python3 -u -m pytest tests/test_solvers.py tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_examples.py -m gpu -x -q --timeout 300 \
  --timeout-method thread -k "pcg or ode or sdirk or c3 or example or solve" > "$O/pytest_c.log" 2>&1 || { tail -30 "$O/pytest_c.log"; exit 1; }
tail -1 "$O/pytest_c.log"
for rep in 1 2; do
  for v in libecm2pa_b.so libecm2pa_c.so; do
    L=cardiac-ablation-ecm2_amd/lib/$v
    timeout -k 10 300 python3 profiles/ab_lib.py $L --workload c3 --steps 20 --warmup 5 --no-cpu-baseline --full-layout 0 > "$O/${v}_$rep.json" 2> "$O/${v}_$rep.err" || { tail -5 "$O/${v}_$rep.err"; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/${v}_$rep.json').read().strip().splitlines()[-1]); p=d['pcg']; print('$v rep $rep', 'Mult', d['ms_per_step'], 'ms; PCG', p['iterations'], 'it', p['seconds'], 's', p['mdof_iter_per_s'], 'MDoF*it/s')"
  done
done
