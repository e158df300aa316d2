#!/bin/bash
# PMC passes over the forward attention kernels: the 64-query kernel (OBST_ATTN_IMPL=3) and the default 32-query one
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
O="$R/gpurun_out/f64pmc"; mkdir -p "$O"
export B=64 KQV=1
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum"
for impl in 3 2; do
  export OBST_ATTN_IMPL=$impl
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $P -d "$O/i${impl}p$i" -o run --output-format csv -- python3 "$R/tools/lab/bench_attn.py" > "$O/i${impl}p$i.log" 2>&1 || { echo "pass $impl/$i failed"; tail -5 "$O/i${impl}p$i.log"; exit 1; }
  done
done
python3 "$R/tools/pmc_summary.py" "$O" > "$O/summary.txt"
grep -A30 "attn_fwd" "$O/summary.txt"
