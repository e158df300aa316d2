set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r6s
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "norm" --timeout 120 --timeout-method thread > gpurun_out/r6s/norm_tests.log 2>&1 || { tail -30 gpurun_out/r6s/norm_tests.log; exit 1; }
tail -1 gpurun_out/r6s/norm_tests.log
for v in old tree f2 f4; do
  if [ $v = tree ]; then unset OBST_KERNELS; else export OBST_KERNELS=$PWD/lab_so/k_$v.so; fi
  timeout -k 10 120 python -u tools/lab/norm_ctx32.py --tag $v >> gpurun_out/r6s/norm_ab.jsonl 2> gpurun_out/r6s/norm_ab_$v.err || exit 1
done
unset OBST_KERNELS
cat gpurun_out/r6s/norm_ab.jsonl
timeout -k 10 300 python -u bench.py --config configs/ctx32_mixer.json --steps 5 --warmup 2 > gpurun_out/r6s/ctx32.log 2>&1 && tail -1 gpurun_out/r6s/ctx32.log | cut -c1-200 && \
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6s/gpu_tests.log 2>&1 && tail -2 gpurun_out/r6s/gpu_tests.log && \
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r6s/bench.log 2>&1 && tail -1 gpurun_out/r6s/bench.log
