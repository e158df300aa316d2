#!/bin/bash
# round 5, second pass: library-free GEMM dispatch (kin / tri 3 on gemm4w), capture probe, bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/r5b
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "gemm or mixer or skinny" > gpurun_out/r5b/kernels.txt 2>&1; rc=$?; echo "kernel tests rc $rc"; tail -3 gpurun_out/r5b/kernels.txt
[ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/r5b/kernels.txt | head -20; exit 1; }
timeout -k 10 200 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_distributed.py -k "graph_capture" > gpurun_out/r5b/capture.txt 2>&1; echo "capture rc $?"; grep -E "ok\"|error_|PASS|FAIL" gpurun_out/r5b/capture.txt | cut -c1-3000 | head -20
timeout -k 10 300 python -u tools/kbench.py mixer --reps 10 > gpurun_out/r5b/mixer.txt 2>&1; echo "mixer rc $?"; cat gpurun_out/r5b/mixer.txt | cut -c1-400
timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r5b/bench.txt 2>&1; echo "bench rc $?"; tail -3 gpurun_out/r5b/bench.txt
