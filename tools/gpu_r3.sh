#!/bin/bash
# Round-3 check: gemm4w harness (stamps), GPU tests, smoke, headline bench on hipBLASLt and on the MFMA kernels.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
F=${GEMM_FILTER:-bf16}
STAMPS=1 SKIP_CHECK=${SKIP_CHECK:-} timeout -k 10 300 bin/gemm_bench 3 5 "$F" > gpurun_out/gemm_bench.log 2>&1 || { echo "gemm_bench failed"; tail -30 gpurun_out/gemm_bench.log; exit 1; }
grep -v "^check" gpurun_out/gemm_bench.log | grep "TF/s\|stamps\|bad" | grep -v " 0/" | head -60
grep "TF/s\|stamps" gpurun_out/gemm_bench.log
[ -n "$GEMM_ONLY" ] && exit 0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/full_gpu.log 2>&1 || { echo "GPU tests failed"; tail -40 gpurun_out/full_gpu.log; exit 1; }
tail -2 gpurun_out/full_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench_lt1.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_lt1.log; exit 1; }
tail -1 gpurun_out/bench_lt1.log
OBST_GEMM_LT=0 timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench_lt0.log 2>&1 || { echo "bench lt0 failed"; tail -20 gpurun_out/bench_lt0.log; exit 1; }
tail -1 gpurun_out/bench_lt0.log
