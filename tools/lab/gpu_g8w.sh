#!/bin/bash
# gemm8w (ping-pong) vs gemm4w vs hipBLASLt: correctness on every shape, then timing (tools/lab/g8w_ab.cpp)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/g8w
timeout -k 10 400 $R/bin/g8w_ab ${ROUNDS:-5} ${REPS:-5} "${FILT:-}" > $R/gpurun_out/g8w/time.txt 2>&1
rc=$?
cat $R/gpurun_out/g8w/time.txt
exit $rc
