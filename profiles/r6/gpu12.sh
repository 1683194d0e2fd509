# round 6, call 12: the gather order of k_apply_tpe_ts, four reps alternating on one box -- slot order (f718aa1,
# libecm2pa_r6b.so), dealt for the write banks everywhere (libecm2pa_r6dealt.so), dealt for lattice-map blocks only
# (libecm2pa_r6c.so = this tree); C4 structured (RM 1) and the reference's numbering (RM 3)
set -o pipefail
O=gpurun_out/r6/gpu12
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_timed_forms.py -k "108" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
A="--variants 0 --full-layout 0 --sdirk 0 --pcg-iters 0 --no-cpu-baseline --steps 100 --warmup 10"
for rep in 1 2 3 4; do
  for v in libecm2pa_r6b.so libecm2pa_r6dealt.so libecm2pa_r6c.so; do
    for num in structured entity; do
      timeout -k 10 300 python3 profiles/ab_lib.py cardiac-ablation-ecm2_amd/lib/$v $A --numbering $num > $O/ab_${v}_${num}_$rep.json 2> $O/ab_${v}_${num}_$rep.err || exit 1
      python3 -c "import json; d=json.loads(open('$O/ab_${v}_${num}_$rep.json').read().strip().splitlines()[-1]); print('$v $num rep $rep', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_avg'])"
    done
  done
done
