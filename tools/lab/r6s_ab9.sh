set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r6s
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -m gpu -x -q -k "gemm or stream or ffn or attention or model or residual or gelu or norm" --timeout 120 --timeout-method thread > gpurun_out/r6s/tpipe2_tests.log 2>&1 || { tail -30 gpurun_out/r6s/tpipe2_tests.log; exit 1; }
tail -1 gpurun_out/r6s/tpipe2_tests.log
for v in tree res0 nodpp; do
  if [ $v = tree ]; then unset OBST_KERNELS; else export OBST_KERNELS=$PWD/lab_so/k_$v.so; fi
  timeout -k 10 120 python -u tools/lab/norm_ctx32.py --tag $v >> gpurun_out/r6s/norm_ab9.jsonl 2>/dev/null || exit 1
done
unset OBST_KERNELS
timeout -k 10 200 python -u tools/lab/epi_side_ab.py >> gpurun_out/r6s/epi_side_ab9.jsonl 2>/dev/null || exit 1
cat gpurun_out/r6s/norm_ab9.jsonl gpurun_out/r6s/epi_side_ab9.jsonl | cut -c1-400
for v in tree zpipe0 tree; do
  if [ $v = tree ]; then unset OBST_KERNELS; else export OBST_KERNELS=$PWD/lab_so/k_$v.so; fi
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r6s/bench_ab9_$v.log 2>&1 || exit 1
  echo "$v $(tail -1 gpurun_out/r6s/bench_ab9_$v.log | cut -c1-140)"
done
