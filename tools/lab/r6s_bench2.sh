set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r6s_last
timeout -k 10 400 python -u bench.py > gpurun_out/r6s_last/bench_default2.log 2>&1 && tail -1 gpurun_out/r6s_last/bench_default2.log | cut -c1-160 && \
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r6s_last/bench_20.log 2>&1 && tail -1 gpurun_out/r6s_last/bench_20.log | cut -c1-160 && \
timeout -k 10 200 python -u tools/kbench.py gemm --reps 10 > gpurun_out/r6s_last/kb_gemm.log 2>&1; grep -h "calib\|fwd d->4d" gpurun_out/r6s_last/kb_gemm.log | head -2 | cut -c1-260
