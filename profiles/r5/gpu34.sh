# round 5, call 34: the summation plan's run order now that the lattice kernels run in XCD-contiguous
# order -- slot order (brick order: each XCD's plan blocks then cover the bricks the same XCD just wrote)
# against the per-form choice (dof / chain order), same box, alternating
set -o pipefail
O=gpurun_out/r5/gpu34
mkdir -p $O
X="--variants 0 --full-layout 0 --no-cpu-baseline --sdirk 0 --pcg-iters 0"
run() {  # tag order bench-args
  local tag=$1 ro=$2; shift 2
  if [ "$ro" = auto ]; then unset ECM2_RUN_ORDER; else export ECM2_RUN_ORDER=$ro; fi
  timeout -k 10 300 python -u bench.py "$@" $X > $O/$tag.json 2> $O/$tag.err || return 1
  python3 -c "import json,sys; b=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=b['roofline']; print(sys.argv[2], b['value'], 'MDoF/s', b['ms_per_step'], 'ms/Mult', 'kernel', r['kernel_ms_avg'], 'rest', round(b['ms_per_step'] - r['kernel_ms_avg'], 5))" $O/$tag.json $tag
}
for rep in 1 2; do
  for ro in auto slot; do
    run c4_${ro}_$rep $ro --workload c4 --steps 50 --warmup 5 &&
    run c4ent_${ro}_$rep $ro --workload c4 --numbering entity --steps 50 --warmup 5 &&
    run c3_${ro}_$rep $ro --workload c3 --steps 30 --warmup 5 || exit 1
  done
done
unset ECM2_RUN_ORDER
