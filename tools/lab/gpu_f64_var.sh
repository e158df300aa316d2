#!/bin/bash
# forward attention timing per kernel-library variant (ab/f64_*.so, OBST_ATTN_IMPL=3) and the 32-query default
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/f64var
export B=64 KQV=1 ONLY=fwd
OBST_ATTN_IMPL=2 timeout -k 10 120 python -u tools/lab/bench_attn.py 2>&1 | grep attn | sed 's/^/impl2 /' || exit 1
for so in ab/f64_*.so; do
  OBST_ATTN_IMPL=3 OBST_KERNELS=$so timeout -k 10 120 python -u tools/lab/bench_attn.py 2>&1 | grep attn | sed "s#^#$so #" || exit 1
done
OBST_ATTN_IMPL=2 timeout -k 10 120 python -u tools/lab/bench_attn.py 2>&1 | grep attn | sed 's/^/impl2 /' || exit 1
