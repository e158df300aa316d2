#!/bin/bash
# GEMM numerics on both paths (MFMA kernels / hipBLASLt), model GPU tests, then the headline bench with and without
# hipBLASLt for the plain GEMMs (each step time-limited)
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for lt in ${LTS:-1 0}; do
  OBST_GEMM_LT=$lt timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_lt$lt.log 2>&1 || { echo "bench lt=$lt failed"; tail -20 gpurun_out/bench_lt$lt.log; exit 1; }
  echo "lt=$lt: $(tail -1 gpurun_out/bench_lt$lt.log)"
done
