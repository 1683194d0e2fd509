# round 5, call 22: the AMDGPU machine-scheduler strategy for the p = 2 kernels (k_tpe.hip built with
# -mllvm --amdgpu-sched-strategy=max-ilp / --amdgpu-use-amdgpu-trackers / --amdgpu-schedule-metric-bias=0
# against the default build): same box, alternating, twice each, on the headline and the drop-in forms
set -o pipefail
L="libecm2pa.so libecm2pa_ilp.so libecm2pa_trk.so libecm2pa_bias.so"
X="--variants 0 --sdirk 0 --pcg-iters 0"
timeout -k 10 900 bash profiles/ab_libs.sh sched_c4 "$L" --workload c4 --steps 50 --warmup 5 $X &&
timeout -k 10 900 bash profiles/ab_libs.sh sched_dropin "$L" --workload c4 --numbering entity --mesh trilinear --geometry-input jacobians --steps 30 --warmup 5 $X
