#!/bin/bash
# per-kernel times of the attention microbenchmark (rocprofv3 kernel trace + stats only)
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
ROOT=$PWD
TAG=${1:-attn}
mkdir -p gpurun_out/prof_$TAG
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/prof_$TAG -o run -- python3 $ROOT/tools/lab/bench_attn.py > $ROOT/gpurun_out/prof_$TAG/bench.log 2>&1 || { echo "prof failed"; tail -20 $ROOT/gpurun_out/prof_$TAG/bench.log; exit 1; }
cd $ROOT
python3 tools/prof_summary.py gpurun_out/prof_$TAG/run_kernel_stats.csv > gpurun_out/prof_$TAG/summary.md
grep attn gpurun_out/prof_$TAG/summary.md
rm -f gpurun_out/prof_$TAG/run_kernel_trace.csv
