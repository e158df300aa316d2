#!/bin/bash
# round 5 full validation, final tree: every GPU test, smoke, headline bench, decode bench, ctx32_mixer
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r5f
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5f/gpu_tests.log 2>&1 || { echo "GPU tests failed"; tail -40 gpurun_out/r5f/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r5f/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5f/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r5f/smoke.log; exit 1; }
tail -1 gpurun_out/r5f/smoke.log
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5f/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/r5f/bench.log; exit 1; }
tail -1 gpurun_out/r5f/bench.log
timeout -k 10 400 python -u tools/bench_decode.py --batch 32 --prompt 512 --new 128 --full-new 0 > gpurun_out/r5f/decode.log 2>&1 || { echo "decode failed"; tail -20 gpurun_out/r5f/decode.log; exit 1; }
grep metric gpurun_out/r5f/decode.log
timeout -k 10 400 python -u bench.py --config configs/ctx32_mixer.json --steps 4 --warmup 2 > gpurun_out/r5f/ctx32.log 2>&1 || { echo "ctx32 bench failed"; tail -20 gpurun_out/r5f/ctx32.log; exit 1; }
tail -1 gpurun_out/r5f/ctx32.log
