#!/bin/bash
# Round-end GPU check: all GPU tests, smoke, the headline bench, the decode bench, the step profile, and the kernel
# perf gate (tools/kbench.py --check profiles/kbench_floor.json: median-of-20 ratios to the same-process calibration;
# KBENCH_WRITE=1 writes a fresh floor file instead of checking).
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
timeout -k 10 400 python -u tools/bench_decode.py --batch 32 --prompt 512 --new 128 --full-new 0 > gpurun_out/decode_final.log 2>&1 || { echo "decode bench failed"; tail -20 gpurun_out/decode_final.log; exit 1; }
grep metric gpurun_out/decode_final.log
bash tools/profile.sh ${PROFILE_TAG:-r5f} --steps 6 --warmup 3 || exit 1
if [ -n "$KBENCH_WRITE" ]; then
  timeout -k 10 600 python -u tools/kbench.py all --write-floors gpurun_out/kbench_floor_new.json > gpurun_out/kbench.log 2>&1
else
  timeout -k 10 600 python -u tools/kbench.py all --check profiles/kbench_floor.json > gpurun_out/kbench.log 2>&1
fi
rc=$?
grep "REGRESSION\|kbench check" gpurun_out/kbench.log
exit $rc
