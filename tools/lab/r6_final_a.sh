#!/bin/bash
# round 6: whole GPU suite + smoke, then the RevNet stream A/B (loss curves + ctx32 step times). usage: OUTDIR
set -o pipefail
out=$1
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    > "$out/full_gpu.log" 2>&1 || { echo "GPU tests failed"; tail -40 "$out/full_gpu.log"; exit 1; }
tail -1 "$out/full_gpu.log"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || { tail -20 "$out/smoke.log"; exit 1; }
tail -1 "$out/smoke.log"
timeout -k 10 900 python -u tools/lab/stream_ab.py > "$out/stream_ab.jsonl" 2>&1 || { tail -20 "$out/stream_ab.jsonl"; exit 1; }
grep '^{' "$out/stream_ab.jsonl"
