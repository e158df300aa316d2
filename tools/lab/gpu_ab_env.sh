#!/bin/bash
# headline bench A/B over one environment variable: VAR=name VALS="a b a b" (back-to-back runs on one box)
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for v in $VALS; do
  env $VAR=$v timeout -k 10 300 python bench.py --steps ${STEPS:-5} --warmup 2 > gpurun_out/bench_ab.log 2>&1 || { echo "bench $VAR=$v failed"; tail -20 gpurun_out/bench_ab.log; exit 1; }
  echo "$VAR=$v: $(tail -1 gpurun_out/bench_ab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
