#!/bin/bash
# gemm4w dynamic tile queue: GEMM / model tests with the queue on, the CU-contention lab (static vs queue), and the
# headline step both ways
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/queue
OBST_G4W_QUEUE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -x -q -k "gemm or forward_backward or linear or token_mixer" --timeout 120 --timeout-method thread > gpurun_out/queue/tests.log 2>&1 || { tail -40 gpurun_out/queue/tests.log; exit 1; }
tail -2 gpurun_out/queue/tests.log
timeout -k 10 120 /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -Icsrc/kernels tools/lab/cu_contention.cpp -o /tmp/cu_contention -Lhomebrewnlp_mtf_amd -l:_kernels.so -Wl,-rpath,$PWD/homebrewnlp_mtf_amd || exit 1
for q in 0 1; do
  OBST_G4W_QUEUE=$q timeout -k 10 120 /tmp/cu_contention > gpurun_out/queue/cu_$q.txt 2>&1 || { cat gpurun_out/queue/cu_$q.txt; exit 1; }
  echo "queue=$q"; cat gpurun_out/queue/cu_$q.txt
done
for q in 1 0; do
  OBST_G4W_QUEUE=$q timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/queue/bench_$q.log 2>&1 || { tail -20 gpurun_out/queue/bench_$q.log; exit 1; }
  echo "queue=$q $(tail -1 gpurun_out/queue/bench_$q.log | cut -c1-220)"
done
