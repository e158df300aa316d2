#!/bin/bash
# round 6: grad zeroing by hipMemsetAsync vs torch fill, 1.3B bench interleaved. usage: OUTDIR
set -o pipefail
out=$1
mkdir -p "$out"
for i in 1 2; do
  for z in 1 0; do
    OBST_ZERO_MEMSET=$z timeout -k 10 400 python -u bench.py > "$out/bench_z${z}_$i.log" 2>&1 || exit 1
    echo "z=$z $(tail -1 "$out/bench_z${z}_$i.log" | cut -c1-200)"
  done
done
timeout -k 10 500 python -u bench.py --config configs/ctx32_mixer.json > "$out/ctx32.log" 2>&1 || exit 1
tail -1 "$out/ctx32.log" | cut -c1-200
