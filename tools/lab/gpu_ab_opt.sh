#!/bin/bash
# norm/optimizer numerics, then the headline bench for several optimizer chunk sizes (each step time-limited)
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -x -q -p no:cacheprovider -k "norm or optim" > gpurun_out/pytest_ab.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/pytest_ab.log; exit 1; }
tail -2 gpurun_out/pytest_ab.log
for c in ${CHUNKS:-65536 262144 1048576}; do
  OBST_OPT_CHUNK=$c timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_c$c.log 2>&1 || { echo "bench $c failed"; tail -20 gpurun_out/bench_c$c.log; exit 1; }
  echo "chunk $c: $(tail -1 gpurun_out/bench_c$c.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
PROF_STEPS=5 bash tools/profile.sh ab --steps 3 --warmup 2
