# round 5, call 29: PMC pins at HEAD after the XCD-contiguous order (sets a, b, c of collect_r5.sh)
set -o pipefail
mkdir -p gpurun_out/r5
for set in a b c; do
  COMMIT=$(cat profiles/r5/COMMIT) timeout -k 10 1000 bash profiles/collect_r5.sh $set > gpurun_out/r5/collect2_$set.txt 2>&1 || { cat gpurun_out/r5/collect2_$set.txt; exit 1; }
  cat gpurun_out/r5/collect2_$set.txt
done
