#!/bin/bash
# Round-end GPU check: all GPU tests, smoke, the headline bench (default = every GEMM on gemm4w, and OBST_GEMM_LT=1 =
# plain products on hipBLASLt, A/B only), step profile, and the
# kernel perf-regression gate (tools/kbench.py --check profiles/kbench_floor.json: exit 1 on a > 5 % regression).
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/full_gpu.log 2>&1 || { echo "GPU tests failed"; tail -40 gpurun_out/full_gpu.log; exit 1; }
tail -2 gpurun_out/full_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_final.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_final.log; exit 1; }
tail -1 gpurun_out/bench_final.log
OBST_GEMM_LT=1 timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench_final_lt1.log 2>&1 || { echo "bench lt1 failed"; tail -20 gpurun_out/bench_final_lt1.log; exit 1; }
tail -1 gpurun_out/bench_final_lt1.log
bash tools/profile.sh ${PROFILE_TAG:-r4f} --steps 6 --warmup 3 || exit 1
timeout -k 10 400 python -u tools/kbench.py all --check profiles/kbench_floor.json > gpurun_out/kbench.log 2>&1
rc=$?
grep "REGRESSION\|kbench check" gpurun_out/kbench.log
exit $rc
