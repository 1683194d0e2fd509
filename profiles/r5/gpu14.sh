# round 5, call 14: PMC pins at HEAD for sets b (c5, c4ent) and c (c4tri, c4enttrijac, c5tri, c3)
set -o pipefail
mkdir -p gpurun_out/r5
COMMIT=$(cat profiles/r5/COMMIT) timeout -k 10 1100 bash profiles/collect_r5.sh b > gpurun_out/r5/collect_b.txt 2>&1 || { cat gpurun_out/r5/collect_b.txt; exit 1; }
cat gpurun_out/r5/collect_b.txt
COMMIT=$(cat profiles/r5/COMMIT) timeout -k 10 1100 bash profiles/collect_r5.sh c > gpurun_out/r5/collect_c.txt 2>&1 || { cat gpurun_out/r5/collect_c.txt; exit 1; }
cat gpurun_out/r5/collect_c.txt
