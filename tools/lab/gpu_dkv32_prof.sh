# dK/dV A/B: the pipelined 32x32 kernel (OBST_ATTN_BWD=2) against the default 16x16 kernel -- attention tests on the
# 32x32 path, then per-kernel times (rocprofv3 kernel trace of tools/kbench.py attn; read the .db with sqlite3)
set -e
mkdir -p gpurun_out
OBST_ATTN_BWD=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "attn or attention" -x -q --timeout 120 --timeout-method thread > gpurun_out/dkv32_tests.log 2>&1
tail -2 gpurun_out/dkv32_tests.log
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bwd1 -o run -- python3 tools/kbench.py attn > gpurun_out/prof_bwd1.log 2>&1
OBST_ATTN_BWD=2 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bwd2 -o run -- python3 tools/kbench.py attn > gpurun_out/prof_bwd2.log 2>&1
grep pflops gpurun_out/prof_bwd1.log gpurun_out/prof_bwd2.log
