#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/r5c
timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_distributed.py -k "graph_capture" > gpurun_out/r5c/capture.txt 2>&1; echo "capture rc $?"; grep -E "PASS|FAIL|\{'part" gpurun_out/r5c/capture.txt | cut -c1-600 | head -20
timeout -k 10 300 python -u tools/kbench.py mixer --reps 10 > gpurun_out/r5c/mixer.txt 2>&1; echo "mixer rc $?"; grep kernel gpurun_out/r5c/mixer.txt | cut -c1-300
timeout -k 10 600 python -u bench.py --config configs/ctx32_mixer.json --steps 6 --warmup 3 > gpurun_out/r5c/ctx32.txt 2>&1; echo "ctx32 rc $?"; tail -2 gpurun_out/r5c/ctx32.txt | cut -c1-400
