#!/bin/bash
# round 6: bf16 gradient streams under fp32 activation streams (revnet_grad_stream_dtype) -- model oracle tests,
# stream A/B (loss curves + ctx32 step time), kbench mixer (auto work order). usage: OUTDIR
set -o pipefail
out=$1
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_model.py \
    -k "forward_backward and mixer" -s > "$out/model_tests.log" 2>&1; echo "model tests exit $?"
grep -E "bf16grad.*rel |passed|failed" "$out/model_tests.log" | tail -24
timeout -k 10 180 python -u tools/kbench.py mixer > "$out/kb_mixer.jsonl" 2>&1 || exit 1
grep tflops "$out/kb_mixer.jsonl" | cut -c1-150
timeout -k 10 1000 python -u tools/lab/stream_ab.py > "$out/stream_ab.jsonl" 2>&1 || { tail -20 "$out/stream_ab.jsonl"; exit 1; }
grep '^{' "$out/stream_ab.jsonl"
