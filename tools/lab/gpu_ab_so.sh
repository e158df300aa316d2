#!/bin/bash
# A/B of the in-tree kernel library against a saved build (ab/_kernels_old.so) on one box: CMD runs with the new
# library, then the old, then the new again (clock drift shows up as a new/new spread).
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
cp homebrewnlp_mtf_amd/_kernels.so ab/_kernels_new.so
for v in new old new; do
  cp ab/_kernels_$v.so homebrewnlp_mtf_amd/_kernels.so
  echo "== $v"
  timeout -k 10 ${TMO:-300} bash -c "$CMD" > gpurun_out/ab_$v.log 2>&1 || { echo "$v failed"; tail -20 gpurun_out/ab_$v.log; exit 1; }
  grep -v "amdgpu.ids" gpurun_out/ab_$v.log | tail -${TAIL:-4}
done
cp ab/_kernels_new.so homebrewnlp_mtf_amd/_kernels.so
