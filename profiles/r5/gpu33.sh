# round 5, call 33: the snapshot kernel without the per-row scheduling barrier (-DECM2_TS_NOSB) against
# the default build, same box, alternating: headline, reference numbering, Pennes
set -o pipefail
L="libecm2pa.so libecm2pa_nosb.so"
X="--variants 0 --sdirk 0 --pcg-iters 0"
timeout -k 10 600 bash profiles/ab_libs.sh nosb_c4 "$L" --workload c4 --steps 50 --warmup 5 $X &&
timeout -k 10 600 bash profiles/ab_libs.sh nosb_c4ent "$L" --workload c4 --numbering entity --steps 50 --warmup 5 $X &&
timeout -k 10 600 bash profiles/ab_libs.sh nosb_pen "$L" --workload c4 --coefficients pennes --steps 50 --warmup 5 $X
