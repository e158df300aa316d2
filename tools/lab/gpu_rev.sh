#!/bin/bash
# fused RevNet stream update: kernel + model tests, then the ctx32_mixer step fused vs unfused
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/rev
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -x -q -k "stream or forward_backward or token_mixer or gemm or norm" --timeout 120 --timeout-method thread > gpurun_out/rev/tests.log 2>&1 || { tail -40 gpurun_out/rev/tests.log; exit 1; }
tail -2 gpurun_out/rev/tests.log
for f in 1 0; do
  OBST_REV_FUSE=$f timeout -k 10 400 python -u bench.py --config configs/ctx32_mixer.json --steps 4 --warmup 2 > gpurun_out/rev/bench_$f.log 2>&1 || { tail -20 gpurun_out/rev/bench_$f.log; exit 1; }
  echo "fuse=$f $(tail -1 gpurun_out/rev/bench_$f.log | cut -c1-200)"
done
