# per-call transpose_kernel durations / grids of the headline step (rocprofv3 kernel trace, .db read with sqlite3)
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/prof_tr -o run -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/prof_tr.log 2>&1
tail -1 gpurun_out/prof_tr.log | cut -c1-120
