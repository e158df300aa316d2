#!/bin/bash
# round 6: work order of the triangular token-mixer products (OBST_G4W_TRI_GROUP: 0 = tile rows slowest, G = batch
# groups) -- oracle tests under G = 8, kbench mixer A/B, ctx32_mixer step A/B, then the aten census. usage: OUTDIR
set -o pipefail
out=$1
mkdir -p "$out"
export TMPDIR=/tmp
OBST_G4W_TRI_GROUP=8 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_kernels.py -k "mixer or tri" > "$out/tests_g8.log" 2>&1 || { tail -30 "$out/tests_g8.log"; exit 1; }
tail -1 "$out/tests_g8.log"
for r in 1 2; do
  for g in 0 8 16 32; do
    OBST_G4W_TRI_GROUP=$g timeout -k 10 180 python -u tools/kbench.py mixer > "$out/kb_mixer_g${g}_r$r.jsonl" 2>&1 || exit 1
    echo "G=$g $(grep -h tflops "$out/kb_mixer_g${g}_r$r.jsonl" | python3 -c 'import sys,json; print([ (json.loads(l)["shape"][6:14], json.loads(l)["us_gemm4w"]) for l in sys.stdin])')"
  done
done
for g in 0 8 32 0 8; do
  OBST_G4W_TRI_GROUP=$g timeout -k 10 400 python -u bench.py --config configs/ctx32_mixer.json --steps 8 --warmup 3 \
      > "$out/ctx32_g$g.log" 2>&1 || exit 1
  echo "ctx32 G=$g $(tail -1 "$out/ctx32_g$g.log" | cut -c100-160)"
done
timeout -k 10 300 python -u tools/lab/aten_census.py --config configs/ctx32_mixer.json --batch 32 \
    > "$out/aten_ctx32.txt" 2>&1 || { tail -20 "$out/aten_ctx32.txt"; exit 1; }
timeout -k 10 300 python -u tools/lab/aten_census.py --config configs/gpt_neo_1.3b.json --batch 8 \
    > "$out/aten_13b.txt" 2>&1 || { tail -20 "$out/aten_13b.txt"; exit 1; }
