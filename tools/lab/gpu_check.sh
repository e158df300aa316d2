#!/bin/bash
# One GPU round: kernel/model tests, smoke, short benches. Each GPU step has its own time limit; stop at the
# first failure (no retries).
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
STAGE=${1:-all}
if [ "$STAGE" = all ] || [ "$STAGE" = tests ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
  tail -3 gpurun_out/pytest_gpu.log
fi
if [ "$STAGE" = all ] || [ "$STAGE" = smoke ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
  tail -2 gpurun_out/smoke.log
fi
if [ "$STAGE" = all ] || [ "$STAGE" = bench ]; then
  timeout -k 10 400 python bench.py --steps 3 --warmup 1 --depth 2 > gpurun_out/bench_d2.log 2>&1 || { echo "bench d2 failed"; tail -30 gpurun_out/bench_d2.log; exit 1; }
  tail -2 gpurun_out/bench_d2.log
  timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench.log; exit 1; }
  tail -2 gpurun_out/bench.log
fi
