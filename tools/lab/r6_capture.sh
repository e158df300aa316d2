#!/bin/bash
# round 6: headline bench on this box, then the RCCL capture probe per part without a launcher (child stderr kept,
# faulthandler, NCCL_DEBUG=INFO). Stops at the first failing step (an abort ends the call).
# usage: tools/lab/r6_capture.sh OUTDIR MODE PART [PART ...]
set -o pipefail
out=$1; mode=$2; shift 2
mkdir -p "$out"
export TMPDIR=/tmp
for part in "$@"; do
  echo "== $part ($mode)" | tee -a "$out/status.txt"
  NCCL_DEBUG=INFO TORCH_SHOW_CPP_STACKTRACES=1 timeout -k 10 150 python -u tools/graph_capture_probe.py \
      --part "$part" --capture-mode "$mode" > "$out/cap_${mode}_${part}.txt" 2>&1
  rc=$?
  echo "$part $mode exit $rc" | tee -a "$out/status.txt"
  tail -5 "$out/cap_${mode}_${part}.txt"
  [ $rc -eq 0 ] || exit $rc
done
