#!/bin/bash
# gemm4w schedule variants vs hipBLASLt (tools/lab/g4w_sched.cpp); usage: tools/lab/gpu_g4w_sched.sh [filter] [tag]
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 bin/g4w_sched 5 5 "${1:-}" > gpurun_out/g4w_sched${2:-}.txt 2>&1
rc=$?
grep -v "^ *$" gpurun_out/g4w_sched${2:-}.txt | grep "TF/s\| [1-9][0-9]*/[0-9]* bad" 
exit $rc
