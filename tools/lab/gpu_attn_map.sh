#!/bin/bash
# attention-map kernels: oracle tests, timings, per-kernel profile
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/amap
[ -n "$SKIP_TESTS" ] || timeout -k 10 300 python -u -m pytest tests/test_gpu_attn_map.py -x -q --timeout 120 --timeout-method thread > gpurun_out/amap/tests.log 2>&1 || { tail -40 gpurun_out/amap/tests.log; exit 1; }
tail -1 gpurun_out/amap/tests.log
timeout -k 10 300 python -u tools/lab/attn_map_lab.py 2>&1 | tee gpurun_out/amap/lab.txt || exit 1
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/amap/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/lab/attn_map_lab.py > $GRAFT_REPO_ROOT/gpurun_out/amap/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/amap/prof.log; exit 1; }
f=$(ls $GRAFT_REPO_ROOT/gpurun_out/amap/prof/*/run_kernel_stats.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(ls $GRAFT_REPO_ROOT/gpurun_out/amap/prof/run_kernel_stats.csv)
cut -d, -f1-5 "$f" | head -12
