#!/bin/bash
# TLAY (row-layout accumulators) validation: GEMM GPU tests (both hipBLASLt legs), then the schedule harness
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/g4w; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "gemm or mixer" > $O/t_kernels.txt 2>&1 || { tail -30 $O/t_kernels.txt; exit 1; }
tail -1 $O/t_kernels.txt
STAMPS=1 SKIP_CHECK=1 timeout -k 10 120 bin/g4w_sched 3 3 "fwd d->2d" > $O/stamps.txt 2>&1 || exit 1
timeout -k 10 500 bin/g4w_sched 3 5 "" > $O/time.txt 2>&1 || exit 1
