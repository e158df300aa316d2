#!/bin/bash
# 64-query forward attention (OBST_ATTN_IMPL=3): numerics vs the fp32 oracle, then A/B timing against the default
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/f64
export OBST_ATTN_IMPL=3
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "attention" --timeout 120 --timeout-method thread > gpurun_out/f64/tests.log 2>&1 || { tail -30 gpurun_out/f64/tests.log; exit 1; }
tail -2 gpurun_out/f64/tests.log
timeout -k 10 200 python -u tools/kbench.py attn > gpurun_out/f64/kb3.log 2>&1 || { tail -20 gpurun_out/f64/kb3.log; exit 1; }
OBST_ATTN_IMPL=2 timeout -k 10 200 python -u tools/kbench.py attn > gpurun_out/f64/kb2.log 2>&1 || { tail -20 gpurun_out/f64/kb2.log; exit 1; }
grep '"attention"' gpurun_out/f64/kb3.log gpurun_out/f64/kb2.log | cut -c1-200
