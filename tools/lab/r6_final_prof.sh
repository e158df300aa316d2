#!/bin/bash
# round 6 (end): step profiles of the final tree (GPT-Neo-1.3B, ctx32_mixer) and the kbench floor check. usage: OUTDIR
set -o pipefail
out=$1
mkdir -p "$out"
export TMPDIR=/tmp
PROF_STEPS=6 bash tools/profile.sh r6e_13b --steps 6 --warmup 3 > /dev/null || exit 1
PROF_STEPS=6 bash tools/profile.sh r6e_ctx32 --config configs/ctx32_mixer.json --steps 6 --warmup 3 > /dev/null || exit 1
timeout -k 10 700 python -u tools/kbench.py all --check profiles/kbench_floor.json > "$out/kbench.log" 2>&1; echo "kbench check exit $?"
grep "REGRESSION\|kbench check" "$out/kbench.log"
exit 0
