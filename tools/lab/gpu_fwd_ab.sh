set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "attn or attention" -x -q --timeout 120 --timeout-method thread > gpurun_out/fwdab_tests.log 2>&1
for i in 1 2; do
  timeout -k 10 120 python -u tools/kbench.py attn >> gpurun_out/fwdab.jsonl 2>&1
  OBST_KERNELS=$PWD/bin/_kernels_nofence.so timeout -k 10 120 python -u tools/kbench.py attn | sed 's/^/nofence /' >> gpurun_out/fwdab.jsonl 2>&1
done
tail -3 gpurun_out/fwdab_tests.log; cat gpurun_out/fwdab.jsonl
