# round 6, call 3: the GPU suite with the energy-folded den (HEAD build), the driver's bench command,
# and a kernel trace of the one-GPU line (the PCG iteration's kernels included)
set -o pipefail
O=gpurun_out/r6/gpu3
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -3 $O/tests.txt
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; b=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('bench', b['value'], b['ms_per_step'], b['roofline']['kernel_ms_avg'], 'drop_in', b['drop_in']['value'], 'entity', b['entity_numbering']['value'], 'pcg', b['pcg_iteration']['iteration_ms'], 'sdirk', b['sdirk_step'])"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --variants 0 --full-layout 0 --sdirk 0 --no-cpu-baseline > $O/prof_bench.json 2> $O/prof_bench.err || { tail -20 $O/prof_bench.err; exit 1; }
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
head -20 $O/kernel_stats.csv
