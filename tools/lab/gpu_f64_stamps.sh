#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../.."
export OBST_ATTN_IMPL=3
for so in ab/f64_stamps.so ab/f64_bare_stamps.so; do for c in 1 0; do
  echo "== $so"; CAUSAL=$c OBST_KERNELS=$so timeout -k 10 120 python -u tools/lab/f64_stamps.py 2>&1 | grep causal || exit 1
done; done
