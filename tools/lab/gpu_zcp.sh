#!/bin/bash
# ctx32_mixer step per stream-update GEMM option variant (ab/zcp_<opt>.so), interleaved twice
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/zcp
for rep in 1 2; do for so in ab/zcp_0.so ab/zcp_2.so ab/zcp_32.so ab/zcp_34.so; do
  OBST_KERNELS=$so timeout -k 10 300 python -u bench.py --config configs/ctx32_mixer.json --steps 3 --warmup 2 > gpurun_out/zcp/b.log 2>&1 || { tail -20 gpurun_out/zcp/b.log; exit 1; }
  echo "$so $(tail -1 gpurun_out/zcp/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done
