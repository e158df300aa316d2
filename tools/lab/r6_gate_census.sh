#!/bin/bash
# round 6: the in-suite perf gate, the RCCL capture tests, an aten-kernel census of the ctx32 step, then the round-5
# all_reduce capture abort reproduced UNDER torchrun with the child's output teed (ends the call if it aborts)
set -o pipefail
out=$1
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/kbench.py norm > "$out/kb_norm.jsonl" 2>&1; timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -s tests/test_gpu_perf_gate.py \
    > "$out/gate.log" 2>&1; echo "gate exit $?"; grep -E "passed|failed|REGRESS|regression" "$out/gate.log" | tail -3
# the deliberately slowed build: the round-1 grid-stride elementwise launch (must FAIL the gate)
OBST_EW_CAP=2048 timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -s \
    tests/test_gpu_perf_gate.py > "$out/gate_slowed.log" 2>&1; echo "slowed gate exit $? (expected 1)"
grep -E "passed|failed|regression" "$out/gate_slowed.log" | tail -2 | cut -c1-300
timeout -k 10 600 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_gpu_distributed.py \
    -k capture > "$out/capture_tests.log" 2>&1 || { tail -30 "$out/capture_tests.log"; exit 1; }
tail -2 "$out/capture_tests.log"
timeout -k 10 300 python -u tools/lab/aten_census.py --config configs/ctx32_mixer.json --batch 32 \
    > "$out/aten_ctx32.txt" 2>&1 || { tail -20 "$out/aten_ctx32.txt"; exit 1; }
timeout -k 10 300 python -u tools/lab/aten_census.py --config configs/gpt_neo_1.3b.json --batch 8 \
    > "$out/aten_13b.txt" 2>&1 || { tail -20 "$out/aten_13b.txt"; exit 1; }
NCCL_DEBUG=INFO TORCH_SHOW_CPP_STACKTRACES=1 timeout -k 10 200 python -m torch.distributed.run --tee 3 \
    --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 tools/graph_capture_probe.py --part all_reduce \
    > "$out/torchrun_all_reduce.txt" 2>&1
echo "torchrun all_reduce exit $?"
