#!/bin/bash
# Round-6 evidence (the kernel whose code changed this round: the coefficient-snapshot
# kernel), one pass per workload, same tree, same box: rocprofv3 kernel-trace stats,
# the FETCH_SIZE and WRITE_SIZE passes (separate: TCC slots), reduced (pmc_reduce.py) and pinned
# with provenance (pmc_pin.py; COMMIT = the tree's commit), then the bench line that reads the pin.
# Usage: COMMIT=<sha> bash profiles/collect_r6.sh <set: a | b | c | d>
#   a: c4 (the headline: structured, affine + the k(T) coefficient snapshot), c4pen (the Pennes operator:
#      both coefficients laws of one field, no per-point stream), c4ex16 (ex16p's M + dt K(u_alpha_gf))
#   b: c4ent (the reference's numbering with the snapshot), c3 (fichera r6)
#   c: the kernels round 6 did not change, re-pinned at the round's final tree: c5 (bricks), c4tri (TRILINEAR
#      lattice kernel), c4enttrijac (the drop-in configuration), c5tri (TRILINEAR_E bricks)
set -uo pipefail
SET=${1:-a}
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/collect_r6
mkdir -p "$O"
export TMPDIR=/tmp PIN_DATE=$(date -u +%Y-%m-%dT%H:%MZ) PIN_SCRIPT=profiles/collect_r6.sh
one() {  # tag layout kernel_key bench-args...
  local tag=$1 layout=$2 key=$3; shift 3
  # (no PCG / SDIRK sub-measurements: their forms run other instantiations of the same kernels,
  # which the PMC passes would average in)
  local args="$* --no-cpu-baseline --full-layout 0 --variants 0 --sdirk 0 --pcg-iters 0"
  local P="$O/prof_$tag"
  mkdir -p "$P"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -d "$P/trace" -o run --output-format csv \
    -- python3 bench.py $args > "$P/bench_trace.json" 2> "$P/trace.err" || return 1
  timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -T -d "$P/fetch" -o run --output-format csv \
    -- python3 bench.py $args > "$P/bench_fetch.json" 2> "$P/fetch.err" || return 1
  timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -T -d "$P/write" -o run --output-format csv \
    -- python3 bench.py $args > "$P/bench_write.json" 2> "$P/write.err" || return 1
  python3 profiles/pmc_reduce.py "$P" > "$P/pmc_summary.json" || return 1
  python3 profiles/pmc_pin.py "$P" "${tag%%_*}" "$key" > "$O/pmc_${tag%%_*}_n1_${layout}.json" || return 1
  cp "$O/pmc_${tag%%_*}_n1_${layout}.json" profiles/
  timeout -k 10 400 python3 bench.py "$@" --variants 0 > "$O/bench_$tag.json" 2> "$O/bench_$tag.err" || return 1
  echo "$tag: $(tail -1 "$O/bench_$tag.json" | cut -c1-160)"
}
if [ "$SET" = a ]; then
  # the headline and the snapshot forms without a per-point stream (k_apply_tpe_ts: padded image, round 6)
  one c4 affine_ts apply --workload c4 --steps 50 --warmup 5 || exit 1
  one c4pen affine_tsm apply --workload c4 --coefficients pennes --steps 50 --warmup 5 || exit 1
  one c4ex16 affine_tsm apply --workload c4 --coefficients ex16 --steps 50 --warmup 5 || exit 1
elif [ "$SET" = d ]; then
  # the brick kernel after its diagonal flux (G = 3)
  one c5 affine_e apply_brick --workload c5 --steps 30 --warmup 5 || exit 1
elif [ "$SET" = c ]; then
  one c5 affine_e apply_brick --workload c5 --steps 30 --warmup 5 || exit 1
  one c4tri trilinear apply --workload c4 --mesh trilinear --steps 30 --warmup 5 || exit 1
  one c4enttrijac trilinear apply --workload c4 --numbering entity --mesh trilinear --geometry-input jacobians --steps 30 --warmup 5 || exit 1
  one c5tri trilinear_e apply_brick --workload c5 --mesh trilinear --steps 30 --warmup 5 || exit 1
else
  # b: the reference's numbering (RM 3: the dealt gather) and configs[2]
  one c4ent affine_ts apply --workload c4 --numbering entity --steps 50 --warmup 5 || exit 1
  one c3 affine_ts apply --workload c3 --steps 30 --warmup 5 || exit 1
fi
