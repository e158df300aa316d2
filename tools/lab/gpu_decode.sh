#!/bin/bash
# GPU check of the serving path: KV-decode tests, decode throughput (graphed / eager / recompute), rocprofv3 stats
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/prof_dec
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_aux.py -k "decode or kv" > gpurun_out/t_dec.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/bench_decode.py --batch 32 --prompt 512 --new 128 --full-new 16 --eager > gpurun_out/dec.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_dec -o dec -- python3 $GRAFT_REPO_ROOT/tools/bench_decode.py --batch 32 --prompt 512 --new 64 --full-new 0 > $GRAFT_REPO_ROOT/gpurun_out/prof_dec/run.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT
STATS=$(find /tmp/prof_dec -name "*kernel_stats.csv" | head -1)
cp "$STATS" gpurun_out/prof_dec/kernel_stats.csv
python3 tools/prof_summary.py "$STATS" 1 > gpurun_out/prof_dec/summary.md
