#!/bin/bash
# Round-4 gemm4w validation: GEMM / mixer / model GPU tests, kbench gemm + mixer, and a same-box A/B of the headline
# bench with hipBLASLt (default) against every GEMM on gemm4w (OBST_GEMM_LT=0).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4g; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "gemm or mixer" > $O/t_kernels.txt 2>&1 || { tail -30 $O/t_kernels.txt; exit 1; }
tail -1 $O/t_kernels.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread -k "forward_backward or fused_optimizer" > $O/t_model.txt 2>&1 || { tail -30 $O/t_model.txt; exit 1; }
tail -1 $O/t_model.txt
timeout -k 10 300 python -u tools/kbench.py gemm > $O/kbench_gemm.jsonl 2>&1 || { tail -5 $O/kbench_gemm.jsonl; exit 1; }
cat $O/kbench_gemm.jsonl
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/bench_lt1_$i.log 2>&1 || { tail -20 $O/bench_lt1_$i.log; exit 1; }
  tail -1 $O/bench_lt1_$i.log | cut -c1-200
  OBST_GEMM_LT=0 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/bench_lt0_$i.log 2>&1 || { tail -20 $O/bench_lt0_$i.log; exit 1; }
  tail -1 $O/bench_lt0_$i.log | cut -c1-200
done
