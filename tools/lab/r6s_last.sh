set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r6s_last
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6s_last/full_gpu.log 2>&1 || { tail -30 gpurun_out/r6s_last/full_gpu.log; exit 1; }
tail -1 gpurun_out/r6s_last/full_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6s_last/smoke.log 2>&1 && tail -1 gpurun_out/r6s_last/smoke.log && \
timeout -k 10 400 python -u bench.py > gpurun_out/r6s_last/bench_default.log 2>&1 && tail -1 gpurun_out/r6s_last/bench_default.log | cut -c1-160
