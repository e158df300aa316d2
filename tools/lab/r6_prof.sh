#!/bin/bash
# round 6: headline bench, step profiles (GPT-Neo-1.3B and ctx32_mixer), kbench (all sections + the floor check),
# decode bench. usage: OUTDIR
set -o pipefail
out=$1
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > "$out/bench.log" 2>&1 || { tail -20 "$out/bench.log"; exit 1; }
tail -1 "$out/bench.log" | cut -c1-200
timeout -k 10 500 python -u bench.py --config configs/ctx32_mixer.json --steps 10 --warmup 3 > "$out/ctx32.log" 2>&1 || { tail -20 "$out/ctx32.log"; exit 1; }
tail -1 "$out/ctx32.log" | cut -c1-200
PROF_STEPS=6 bash tools/profile.sh r6_13b --steps 6 --warmup 3 > /dev/null || exit 1
PROF_STEPS=6 bash tools/profile.sh r6_ctx32 --config configs/ctx32_mixer.json --steps 6 --warmup 3 > /dev/null || exit 1
cp -r gpurun_out/prof_r6_13b gpurun_out/prof_r6_ctx32 "$out/" 2>/dev/null
timeout -k 10 700 python -u tools/kbench.py all --check profiles/kbench_floor.json > "$out/kbench.log" 2>&1; echo "kbench check exit $?"
grep "REGRESSION\|kbench check" "$out/kbench.log"
