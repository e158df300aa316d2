#!/bin/bash
# forward attention, 64-query kernel (impl 3) vs the default (impl 2): causal and full, two batch sizes
set -o pipefail
cd "$(dirname "$0")/../.."
export KQV=1 ONLY=fwd
for c in 0 1; do for b in 16 64; do for impl in 2 3; do
  CAUSAL=$c B=$b OBST_ATTN_IMPL=$impl timeout -k 10 120 python -u tools/lab/bench_attn.py 2>&1 | grep attn | sed "s/^/impl$impl /" || exit 1
done; done; done
