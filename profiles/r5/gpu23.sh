# round 5, call 23: nontemporal y / partial stores in the p = 2 kernels' final store (-DECM2_NT_STORES)
# against the default build, same box, alternating: headline, reference numbering, drop-in
set -o pipefail
L="libecm2pa.so libecm2pa_nt.so"
X="--variants 0 --sdirk 0 --pcg-iters 0"
timeout -k 10 600 bash profiles/ab_libs.sh nt_c4 "$L" --workload c4 --steps 50 --warmup 5 $X &&
timeout -k 10 600 bash profiles/ab_libs.sh nt_c4ent "$L" --workload c4 --numbering entity --steps 50 --warmup 5 $X &&
timeout -k 10 600 bash profiles/ab_libs.sh nt_dropin "$L" --workload c4 --numbering entity --mesh trilinear --geometry-input jacobians --steps 30 --warmup 5 $X
