# round 5, call 28: the XCD-contiguous order adopted in the lattice kernels -- parity (whole GPU parity
# and timed-form files), then the same order for k_apply_tpe_sf (-DECM2_SF_XCD) A/B: C4 without the
# snapshot (sf RM 1) and the N = 8 member emulation (sf on partitioned forms)
set -o pipefail
O=gpurun_out/r5/gpu28
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_timed_forms.py tests/test_gpu_snapshot_laws.py > $O/parity.txt 2>&1 || { tail -30 $O/parity.txt; exit 1; }
tail -1 $O/parity.txt
L="libecm2pa.so libecm2pa_sfx.so"
X="--variants 0 --sdirk 0 --pcg-iters 0"
timeout -k 10 600 bash profiles/ab_libs.sh sfx_c4 "$L" --workload c4 --coefficient-snapshot 0 --steps 50 --warmup 5 $X || exit 1
for rep in 1 2; do
  for v in libecm2pa.so libecm2pa_sfx.so; do
    timeout -k 10 300 python3 profiles/ab_lib.py cardiac-ablation-ecm2_amd/lib/$v --workload c4 --loopback 8 --member -1 \
      --steps 50 --warmup 5 --no-cpu-baseline --full-layout 0 > $O/member_${v}_$rep.json 2> $O/member_${v}_$rep.err || exit 1
    python3 -c "import json,sys; b=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'N=8 slowest', b['slowest_member_ms'], b['member_ms'])" $O/member_${v}_$rep.json "$v rep $rep"
  done
done
