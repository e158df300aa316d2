#!/bin/bash
# round 6: GPU model tests incl. the bf16 RevNet stream variants, the capture tests (watchdog quiesce), the RevNet
# stream dtype A/B on ctx32_mixer (loss curves + step time), the aten census, then the round-5 all_reduce capture
# UNDER torchrun with the child's output teed (last: ends the call if it aborts). usage: OUTDIR
set -o pipefail
out=$1
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_model.py \
    -k "forward_backward" -s > "$out/model_tests.log" 2>&1; grep -E "rel |passed|failed" "$out/model_tests.log" | tail -40
tail -1 "$out/model_tests.log"
timeout -k 10 600 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_gpu_distributed.py \
    -k capture > "$out/capture_tests.log" 2>&1 || { grep -E "PASS|FAIL" "$out/capture_tests.log"; exit 1; }
grep -E "PASS|FAIL" "$out/capture_tests.log"
timeout -k 10 900 python -u tools/lab/stream_ab.py > "$out/stream_ab.jsonl" 2>&1 || { tail -20 "$out/stream_ab.jsonl"; exit 1; }
grep '^{' "$out/stream_ab.jsonl"
timeout -k 10 300 python -u tools/lab/aten_census.py --config configs/ctx32_mixer.json --batch 32 \
    > "$out/aten_ctx32.txt" 2>&1 || { tail -20 "$out/aten_ctx32.txt"; exit 1; }
timeout -k 10 300 python -u tools/lab/aten_census.py --config configs/gpt_neo_1.3b.json --batch 8 \
    > "$out/aten_13b.txt" 2>&1 || { tail -20 "$out/aten_13b.txt"; exit 1; }
NCCL_DEBUG=INFO TORCH_SHOW_CPP_STACKTRACES=1 timeout -k 10 200 python -m torch.distributed.run --tee 3 \
    --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 tools/graph_capture_probe.py --part all_reduce \
    --capture-mode global > "$out/torchrun_all_reduce.txt" 2>&1
echo "torchrun all_reduce exit $?"
