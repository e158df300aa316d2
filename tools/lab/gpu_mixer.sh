#!/bin/bash
# 32ctx_mixer (config 3 of BASELINE.json) per-GPU throughput at its DP=8 per-GPU batch of 32
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 500 python bench.py --config configs/ctx32_mixer.json --batch-per-gpu 32 --steps 3 --warmup 2 > gpurun_out/bench_mixer.log 2>&1 || { tail -20 gpurun_out/bench_mixer.log; exit 1; }
tail -1 gpurun_out/bench_mixer.log
