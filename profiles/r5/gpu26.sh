# round 5, call 26: configs[2] (fichera r6, the reference's numbering) and configs[4] (C5) with the
# Pennes operator (perfusion law of T as the mass, k(T) diffusion) and ex16p's coefficients
set -o pipefail
O=gpurun_out/r5/gpu26
mkdir -p $O
for wl in c3 c5; do
  for cf in pennes ex16; do
    timeout -k 10 400 python -u bench.py --workload $wl --coefficients $cf --steps 30 --warmup 5 --variants 0 \
      --full-layout 0 --no-cpu-baseline > $O/${wl}_$cf.json 2> $O/${wl}_$cf.err || { tail -20 $O/${wl}_$cf.err; exit 1; }
    python3 -c "
import json; b = json.loads(open('$O/${wl}_$cf.json').read().strip().splitlines()[-1])
print('$wl $cf', b['value'], 'MDoF/s', b['ms_per_step'], 'ms', b['config']['qdata_layout'], 'kernel', b['roofline']['kernel_ms_avg'], 'pcg', (b.get('pcg') or {}).get('mdof_iter_per_s'), 'sdirk', (b.get('sdirk_step') or {}).get('step_ms'))"
  done
done
