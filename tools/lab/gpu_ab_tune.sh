#!/bin/bash
# headline bench A/B of hipBLASLt candidate tuning (same process image, back-to-back runs)
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for t in ${TUNES:-0 1 0 1}; do
  OBST_LT_TUNE=$t timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_tune$t.log 2>&1 || { echo "bench tune=$t failed"; tail -20 gpurun_out/bench_tune$t.log; exit 1; }
  echo "tune=$t: $(tail -1 gpurun_out/bench_tune$t.log | cut -c1-140)"
done
