# round 5: PMC pins at HEAD (set a: the headline, the Pennes and ex16 snapshot forms)
set -o pipefail
mkdir -p gpurun_out/r5
COMMIT=$(cat profiles/r5/COMMIT) timeout -k 10 1100 bash profiles/collect_r5.sh a > gpurun_out/r5/collect_a.txt 2>&1
