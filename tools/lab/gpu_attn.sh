#!/bin/bash
# attention numerics + A/B throughput of the attention kernel generations (each step time-limited)
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -x -q -p no:cacheprovider -k attention > gpurun_out/pytest_attn.log 2>&1 || { echo "attention tests failed"; tail -40 gpurun_out/pytest_attn.log; exit 1; }
tail -2 gpurun_out/pytest_attn.log
for impl in ${IMPLS:-1 2}; do
  OBST_ATTN_IMPL=$impl timeout -k 10 120 python tools/lab/bench_attn.py > gpurun_out/bench_attn_$impl.log 2>&1 || { echo "bench_attn $impl failed"; tail -20 gpurun_out/bench_attn_$impl.log; exit 1; }
  echo "impl $impl"; cat gpurun_out/bench_attn_$impl.log
done
