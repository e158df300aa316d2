#!/bin/bash
# PMC counters (two passes, kernel trace only) of the kernels matching KREGEX while running a python tool:
#   TAG=name KREGEX=regex pmc_cmd.sh tools/lab/bench_norm.py [args]
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
ROOT=$PWD
TAG=${TAG:-cmd}
mkdir -p gpurun_out/pmc_$TAG
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_WAVES"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $ROOT/gpurun_out/pmc_$TAG/p$i \
    --kernel-include-regex "$KREGEX" -- python3 $ROOT/"$@" > $ROOT/gpurun_out/pmc_$TAG/p$i.log 2>&1 \
    || { echo "pass $i failed"; tail -20 $ROOT/gpurun_out/pmc_$TAG/p$i.log; exit 1; }
done
python3 $ROOT/tools/pmc_summary.py $ROOT/gpurun_out/pmc_$TAG > $ROOT/gpurun_out/pmc_$TAG/summary.txt
cat $ROOT/gpurun_out/pmc_$TAG/summary.txt
