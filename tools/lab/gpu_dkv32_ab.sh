# dK/dV A/B: the software-pipelined 32x32 kernel (OBST_ATTN_BWD=2) against the default 16x16 kernel
set -e
mkdir -p gpurun_out
OBST_ATTN_BWD=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "attn or attention" -x -q --timeout 120 --timeout-method thread > gpurun_out/dkv32_tests.log 2>&1
for i in 1 2; do
  timeout -k 10 120 python -u tools/kbench.py attn | sed 's/^/bwd1 /' >> gpurun_out/dkv32.jsonl 2>&1
  OBST_ATTN_BWD=2 timeout -k 10 120 python -u tools/kbench.py attn | sed 's/^/bwd2 /' >> gpurun_out/dkv32.jsonl 2>&1
done
tail -3 gpurun_out/dkv32_tests.log; cat gpurun_out/dkv32.jsonl
