# round 6, call 24: the diagonal flux product of the snapshot kernel on axis-aligned meshes
# (k_apply_tpe_ts<..., CD>, FluxDiagonal) -- parity, then the C4 headline / reference numbering / Pennes
# Mult against ECM2_CDIAG=0 (the general product) on the same box
set -o pipefail
O=gpurun_out/r6/gpu24
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_timed_forms.py \
  tests/test_gpu_parity.py tests/test_gpu_configs.py -k "snapshot or diagonal or c4 or timed or energy or law or pennes or ex16" \
  > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
A="--variants 0 --full-layout 0 --sdirk 0 --no-cpu-baseline --steps 40 --warmup 5 --pcg-iters 20"
for rep in 1 2; do
  for c in 1 0; do
    for w in "--workload c4" "--workload c4 --numbering entity" "--workload c4 --coefficients pennes"; do
      t=$(echo "$w" | tr -d ' -')
      ECM2_CDIAG=$c timeout -k 10 300 python3 bench.py $A $w > $O/${t}_cd${c}_$rep.json 2> $O/${t}_cd${c}_$rep.err || exit 1
      python3 -c "import json; d=json.loads(open('$O/${t}_cd${c}_$rep.json').read().strip().splitlines()[-1]); print('cdiag=$c rep $rep $t', d['value'], d['ms_per_step'], 'kernel', d['roofline']['kernel_ms_avg'], 'pcg', d['pcg_iteration']['iteration_ms'])"
    done
  done
done
