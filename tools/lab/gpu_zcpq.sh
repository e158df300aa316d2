#!/bin/bash
# queued fp32 + bf16-copy GEMMs: kernel tests, then ctx32_mixer with the tile queue on / off / on (one box)
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/zcpq
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -x -q -k "stream or gemm or forward_backward or token_mixer" --timeout 120 --timeout-method thread > gpurun_out/zcpq/tests.log 2>&1 || { tail -30 gpurun_out/zcpq/tests.log; exit 1; }
tail -1 gpurun_out/zcpq/tests.log
for q in 1 0 1; do
  OBST_G4W_QUEUE=$q timeout -k 10 400 python -u bench.py --config configs/ctx32_mixer.json --steps 4 --warmup 2 > gpurun_out/zcpq/ctx32_$q.log 2>&1 || { tail -20 gpurun_out/zcpq/ctx32_$q.log; exit 1; }
  echo "queue=$q $(tail -1 gpurun_out/zcpq/ctx32_$q.log | cut -c1-150)"
done
