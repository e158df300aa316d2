set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r6s
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -m gpu -x -q -k "stream or revnet or norm or sink or mixer or gemm" --timeout 120 --timeout-method thread > gpurun_out/r6s/z2_tests.log 2>&1 || { tail -30 gpurun_out/r6s/z2_tests.log; exit 1; }
tail -1 gpurun_out/r6s/z2_tests.log
for v in tree zpipe0 tree; do
  if [ $v = tree ]; then unset OBST_KERNELS; else export OBST_KERNELS=$PWD/lab_so/k_$v.so; fi
  timeout -k 10 300 python -u bench.py --config configs/ctx32_mixer.json --steps 5 --warmup 2 > gpurun_out/r6s/ctx32_ab10_$v.log 2>&1 || exit 1
  echo "$v $(tail -1 gpurun_out/r6s/ctx32_ab10_$v.log | cut -c1-140)"
done
unset OBST_KERNELS
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r6s/bench_ab10.log 2>&1 && tail -1 gpurun_out/r6s/bench_ab10.log | cut -c1-140
