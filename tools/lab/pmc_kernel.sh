#!/bin/bash
# PMC counters of the kernels matching KREGEX during a short bench run (4 passes, kernel trace only; each pass
# within the per-block counter limits; PYARGS: another python program + args under the repo root)
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
ROOT=$PWD
TAG=${TAG:-k}
mkdir -p gpurun_out/pmc_$TAG
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_WAVES"
P2="SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE"
P3="FETCH_SIZE TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"
P4="WRITE_SIZE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_MFMA"
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $ROOT/gpurun_out/pmc_$TAG/p$i \
    --kernel-include-regex "$KREGEX" -- python3 $ROOT/${PYARGS:-bench.py --steps 1 --warmup 1} > $ROOT/gpurun_out/pmc_$TAG/p$i.log 2>&1 \
    || { echo "pass $i failed"; tail -20 $ROOT/gpurun_out/pmc_$TAG/p$i.log; exit 1; }
  find $ROOT/gpurun_out/pmc_$TAG/p$i -name "*kernel_trace.csv" -delete
done
python3 $ROOT/tools/pmc_summary.py $ROOT/gpurun_out/pmc_$TAG > $ROOT/gpurun_out/pmc_$TAG/summary.txt
cat $ROOT/gpurun_out/pmc_$TAG/summary.txt
