# round 5, call 32: XCD-chunked workgroup order (XCD x takes chunks of K = 16 / 64 consecutive brick
# groups in turn) against the adopted fully contiguous ranges, lattice kernels, same box, alternating
set -o pipefail
L="libecm2pa.so libecm2pa_ch16.so libecm2pa_ch64.so"
X="--variants 0 --sdirk 0 --pcg-iters 0"
timeout -k 10 600 bash profiles/ab_libs.sh ch_c4 "$L" --workload c4 --steps 50 --warmup 5 $X &&
timeout -k 10 600 bash profiles/ab_libs.sh ch_c4ent "$L" --workload c4 --numbering entity --steps 50 --warmup 5 $X &&
timeout -k 10 600 bash profiles/ab_libs.sh ch_dropin "$L" --workload c4 --numbering entity --mesh trilinear --geometry-input jacobians --steps 30 --warmup 5 $X
