# round 6, call 28: the diagonal flux in the p = 4 brick kernel (k_apply_brick_c G = 3 on axis-aligned AFFINE_E forms) --
# parity, then the C5 Mult against ECM2_CDIAG=0 on the same box
set -o pipefail
O=gpurun_out/r6/gpu28
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_timed_forms.py \
  tests/test_gpu_configs.py tests/test_gpu_parity.py -k "diagonal or c5 or brick or line or p4" \
  > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
A="--workload c5 --variants 0 --full-layout 0 --sdirk 0 --no-cpu-baseline --steps 40 --warmup 5 --pcg-iters 20"
for rep in 1 2; do
  for c in 1 0; do
    ECM2_CDIAG=$c timeout -k 10 300 python3 bench.py $A > $O/c5_cd${c}_$rep.json 2> $O/c5_cd${c}_$rep.err || exit 1
    python3 -c "import json; d=json.loads(open('$O/c5_cd${c}_$rep.json').read().strip().splitlines()[-1]); print('cdiag=$c rep $rep', d['value'], d['ms_per_step'], 'kernel', d['roofline']['kernel_ms_avg'], 'pcg', d['pcg_iteration']['iteration_ms'])"
  done
done
