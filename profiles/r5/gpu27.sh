# round 5, call 27: XCD-contiguous workgroup order in the p = 2 lattice kernels (-DECM2_TPE_XCD: consecutive
# Morton brick groups on one XCD's L2) against the default round-robin dispatch, same box, alternating
set -o pipefail
L="libecm2pa.so libecm2pa_xcd.so"
X="--variants 0 --sdirk 0 --pcg-iters 0"
timeout -k 10 600 bash profiles/ab_libs.sh xcd_c4 "$L" --workload c4 --steps 50 --warmup 5 $X &&
timeout -k 10 600 bash profiles/ab_libs.sh xcd_c4ent "$L" --workload c4 --numbering entity --steps 50 --warmup 5 $X &&
timeout -k 10 600 bash profiles/ab_libs.sh xcd_dropin "$L" --workload c4 --numbering entity --mesh trilinear --geometry-input jacobians --steps 30 --warmup 5 $X
