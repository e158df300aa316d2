#!/bin/bash
# queue-aware split-K doubling (OBST_G4W_QSPLIT): GEMM tests, then the headline step on / off / on (one box)
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/qsplit
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "gemm or splitk or queue" --timeout 120 --timeout-method thread > gpurun_out/qsplit/tests.log 2>&1 || { tail -30 gpurun_out/qsplit/tests.log; exit 1; }
tail -1 gpurun_out/qsplit/tests.log
for q in 1 0 1; do
  OBST_G4W_QSPLIT=$q timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/qsplit/bench_$q.log 2>&1 || { tail -20 gpurun_out/qsplit/bench_$q.log; exit 1; }
  echo "qsplit=$q $(tail -1 gpurun_out/qsplit/bench_$q.log | cut -c1-150)"
done
