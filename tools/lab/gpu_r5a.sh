#!/bin/bash
# round 5, first GPU pass: gemm8w A/B, the new DP-wire / capture tests, the rewritten skinny decode kernel
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/r5a
bash tools/lab/gpu_g8w.sh > gpurun_out/r5a/g8w.txt 2>&1; echo "g8w rc $?"
grep -E "bad|TF/s" gpurun_out/r5a/g8w.txt | head -80
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "skinny" > gpurun_out/r5a/skinny.txt 2>&1; echo "skinny tests rc $?"
tail -5 gpurun_out/r5a/skinny.txt
timeout -k 10 300 python -u tools/bench_decode.py --batch 32 --prompt 512 --new 128 --full-new 0 > gpurun_out/r5a/dec.txt 2>&1; echo "decode rc $?"
grep metric gpurun_out/r5a/dec.txt
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_distributed.py -k "graph_capture or dp_matches or two_rank" > gpurun_out/r5a/dist.txt 2>&1; echo "dist rc $?"
grep -E "PASS|FAIL|Error|ok\"" gpurun_out/r5a/dist.txt | head -20
