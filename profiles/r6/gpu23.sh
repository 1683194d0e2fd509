# round 6, call 23: the fused cooperative PCG step (k_pcg_fused: step_r + test + update_xd, z in registers / LDS,
# 8 streams) -- PCG / SDIRK parity, then the C4 marginal PCG iteration against ECM2_PCG_FUSED=0 on the same box,
# and its kernel trace
set -o pipefail
O=gpurun_out/r6/gpu23
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_solvers.py tests/test_gpu_configs.py tests/test_gpu_bench_rank_path.py -k "pcg or PCG or ode or sdirk or solve or heat or c3" \
  > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
A="--variants 0 --full-layout 0 --sdirk 0 --no-cpu-baseline --steps 30 --warmup 5 --pcg-iters 20"
for rep in 1 2; do
  for f in 1 0; do
    ECM2_PCG_FUSED=$f timeout -k 10 300 python3 bench.py $A --workload c4 > $O/c4_f${f}_$rep.json 2> $O/c4_f${f}_$rep.err || exit 1
    python3 -c "import json; d=json.loads(open('$O/c4_f${f}_$rep.json').read().strip().splitlines()[-1]); print('fused=$f rep $rep', d['value'], d['ms_per_step'], 'pcg_it_ms', d['pcg_iteration']['iteration_ms'])"
  done
done
exit 0
