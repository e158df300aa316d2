#!/bin/bash
# flash attention built with VGPR-form MFMAs (ab/attn_vgpr.so) vs the default library: tests, interleaved kbench
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/avg
OBST_KERNELS=$PWD/ab/attn_vgpr.so timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "attention" --timeout 120 --timeout-method thread > gpurun_out/avg/tests.log 2>&1 || { tail -30 gpurun_out/avg/tests.log; exit 1; }
tail -1 gpurun_out/avg/tests.log
for v in default vgpr default vgpr; do
  if [ $v = vgpr ]; then export OBST_KERNELS=$PWD/ab/attn_vgpr.so; else unset OBST_KERNELS; fi
  timeout -k 10 200 python -u tools/kbench.py attn 2>/dev/null | grep '"attention"' | cut -c1-170 | sed "s/^/$v /" || exit 1
done
