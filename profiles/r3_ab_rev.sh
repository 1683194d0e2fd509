#!/bin/bash
# Same-box A/B: the TPE apply kernel's workgroups dispatched in reverse block order (c: the rank's
# map-addressed ghost-touching / leftover blocks first, the lattice-addressed interior in the tail)
# against launch order (b), on the emulated per-rank Mult (bench.py --loopback N --member -1) and N = 1.
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r3rev
mkdir -p "$O"
export TMPDIR=/tmp
for rep in 1 2; do
  for v in libecm2pa_b.so libecm2pa_c.so; do
    for N in 1 2 4 8; do
      M=""; [ $N -gt 1 ] && M="--loopback $N --member -1"
      timeout -k 10 300 python3 profiles/ab_lib.py cardiac-ablation-ecm2_amd/lib/$v --workload c4 --steps 50 --warmup 5 \
        --no-cpu-baseline --full-layout 0 --variants 0 $M > "$O/${v}_n${N}_$rep.json" 2> "$O/${v}_n${N}_$rep.err" || { tail -5 "$O/${v}_n${N}_$rep.err"; exit 1; }
      python3 -c "import json,sys; b=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'N=%s' % b.get('emulated_n_gpus', 1), b.get('emulated_value', b.get('value')), 'MDoF/s slowest', b.get('slowest_member_ms', b.get('ms_per_step')), 'ms', b.get('member_ms', ''))" "$O/${v}_n${N}_$rep.json" "$v rep $rep"
    done
  done
done
