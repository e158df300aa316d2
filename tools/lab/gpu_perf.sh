#!/bin/bash
# GPU numerics for the GEMM/model paths, then kernel microbenchmarks and the headline bench (each step time-limited).
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 200 python tools/lab/bench_gemm.py > gpurun_out/bench_gemm.log 2>&1 || { echo "bench_gemm failed"; tail -20 gpurun_out/bench_gemm.log; exit 1; }
cat gpurun_out/bench_gemm.log
timeout -k 10 120 python tools/lab/bench_attn.py > gpurun_out/bench_attn.log 2>&1 || { echo "bench_attn failed"; tail -20 gpurun_out/bench_attn.log; exit 1; }
cat gpurun_out/bench_attn.log
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
