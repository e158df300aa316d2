#!/bin/bash
# PMC counters of the attention kernels (two passes; counter collection only with --kernel-trace, no other traces)
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
ROOT=$PWD
mkdir -p gpurun_out/pmc_attn
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $ROOT/gpurun_out/pmc_attn/counters.txt 2>&1 || true
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES"
P2="SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $ROOT/gpurun_out/pmc_attn/p$i \
    --kernel-include-regex "${KREGEX:-attn_}" -- python3 $ROOT/tools/lab/bench_attn.py > $ROOT/gpurun_out/pmc_attn/p$i.log 2>&1 \
    || { echo "pass $i failed"; tail -20 $ROOT/gpurun_out/pmc_attn/p$i.log; exit 1; }
done
python3 $ROOT/tools/pmc_summary.py $ROOT/gpurun_out/pmc_attn > $ROOT/gpurun_out/pmc_attn/summary.txt
cat $ROOT/gpurun_out/pmc_attn/summary.txt
