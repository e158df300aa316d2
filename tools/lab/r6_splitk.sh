#!/bin/bash
# round 6: split-K for long-K many-tile fp32 products (the logits weight gradient), bf16-stream model tests (fused
# and unfused), gate, headline bench. usage: OUTDIR
set -o pipefail
out=$1
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py \
    -k "splitk or wgrad or queue" > "$out/gemm_tests.log" 2>&1 || { tail -30 "$out/gemm_tests.log"; exit 1; }
tail -1 "$out/gemm_tests.log"
timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_model.py \
    -k "forward_backward and bf16stream" -s > "$out/model_tests.log" 2>&1; echo "model tests exit $?"
grep -E "rel |passed|failed" "$out/model_tests.log" | tail -40
timeout -k 10 300 python -u tools/kbench.py gemm > "$out/kb_gemm.jsonl" 2>&1 || exit 1
grep logits "$out/kb_gemm.jsonl" | cut -c1-200
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -s tests/test_gpu_perf_gate.py \
    > "$out/gate.log" 2>&1; echo "gate exit $?"
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > "$out/bench.log" 2>&1 || exit 1
tail -1 "$out/bench.log" | cut -c1-200
