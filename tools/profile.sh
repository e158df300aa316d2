#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run; summary CSV lands in gpurun_out/prof_<tag>/
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG=${1:-d2}; shift
mkdir -p gpurun_out/prof_$TAG
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run -- python3 $GRAFT_REPO_ROOT/bench.py "$@" > $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG/bench.log 2>&1
rc=$?
cd $GRAFT_REPO_ROOT
STATS=$(find gpurun_out/prof_$TAG -name "*kernel_stats.csv" | head -1)
python3 tools/prof_summary.py "$STATS" ${PROF_STEPS:-1} > gpurun_out/prof_$TAG/summary.md
TRACE=$(find gpurun_out/prof_$TAG -name "*kernel_trace.csv" | head -1)
python3 tools/prof_steps.py "$TRACE" > gpurun_out/prof_$TAG/steps.md && head -30 gpurun_out/prof_$TAG/steps.md
[ -n "$PROF_SEQ" ] && python3 tools/prof_seq.py "$TRACE" > gpurun_out/prof_$TAG/seq.txt
find gpurun_out/prof_$TAG -name "*kernel_trace.csv" -delete
exit $rc
