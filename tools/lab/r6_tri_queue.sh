#!/bin/bash
# round 6: triangular (token-mixer) products on the gemm4w tile queue -- GPU oracle tests, kbench mixer A/B
# (OBST_G4W_QUEUE_TRI 0 / 1 interleaved), ctx32_mixer step A/B. usage: tools/lab/r6_tri_queue.sh OUTDIR
set -o pipefail
out=$1
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
    -k "attention or attn or mixer or queue or tri" > "$out/tests.log" 2>&1 || { tail -30 "$out/tests.log"; exit 1; }
tail -2 "$out/tests.log"
for r in 1 2; do
  for q in 1 0; do
    OBST_G4W_QUEUE_TRI=$q timeout -k 10 180 python -u tools/kbench.py mixer >> "$out/kb_mixer_q$q.jsonl" 2>&1 || exit 1
  done
done
grep -h tflops "$out"/kb_mixer_q*.jsonl | cut -c1-160
for q in 1 0; do
  OBST_G4W_QUEUE_TRI=$q timeout -k 10 400 python -u bench.py --config configs/ctx32_mixer.json --steps 10 --warmup 3 \
      > "$out/ctx32_q$q.log" 2>&1 || exit 1
  tail -1 "$out/ctx32_q$q.log" | cut -c1-200
done
