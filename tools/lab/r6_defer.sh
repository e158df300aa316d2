#!/bin/bash
# round 6: gemm4w DEFER (half... a quarter of each tile's C stores issued in the next tile's first K-tile) --
# GEMM oracle tests, kbench gemm A/B (OBST_G4W_DEFER 1 / 0 interleaved), headline bench A/B. usage: OUTDIR
set -o pipefail
out=$1
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
    -k "gemm or queue or mixer or linear" > "$out/tests.log" 2>&1 || { tail -30 "$out/tests.log"; exit 1; }
tail -1 "$out/tests.log"
for r in 1 2; do
  for d in 1 0; do
    OBST_G4W_DEFER=$d timeout -k 10 300 python -u tools/kbench.py gemm >> "$out/kb_gemm_d$d.jsonl" 2>&1 || exit 1
  done
done
for d in 1 0 1 0; do
  OBST_G4W_DEFER=$d timeout -k 10 400 python -u bench.py --steps 15 --warmup 4 > "$out/bench_d$d.log" 2>&1 || exit 1
  echo "defer=$d $(tail -1 "$out/bench_d$d.log" | cut -c1-140)"
done
