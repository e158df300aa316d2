#!/bin/bash
# headline step, tile queue on / off / on (one box), then the step profile of the default tree
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/qab
for q in 1 0 1; do
  OBST_G4W_QUEUE=$q timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/qab/bench_$q.log 2>&1 || { tail -20 gpurun_out/qab/bench_$q.log; exit 1; }
  echo "queue=$q $(tail -1 gpurun_out/qab/bench_$q.log | cut -c1-160)"
done
bash tools/profile.sh r5f --steps 4 --warmup 2
