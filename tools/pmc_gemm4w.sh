#!/bin/bash
# PMC passes over one GEMM shape of bin/gemm_bench (hipBLASLt, phase and gemm4w kernels in one process).
# usage: tools/pmc_gemm4w.sh <shape filter> <outdir>
set -e
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
F="$1"; O="$R/$2"; mkdir -p "$O"
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum"
P3="TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TA_BUSY_avr TA_TA_BUSY_sum"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  SKIP_CHECK=1 timeout -s KILL 120 rocprofv3 --pmc $P -d "$O/p$i" -o run --output-format csv -- "$R/bin/gemm_bench" 1 3 "$F" > "$O/p$i.log" 2>&1 || echo "pass $i failed"
done
python3 "$R/tools/pmc_summary.py" "$O" > "$O/summary.txt"
echo done
