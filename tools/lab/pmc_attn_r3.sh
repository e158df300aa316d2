# PMC passes (one per run, kernel-trace implied) over tools/kbench.py attn: MFMA busy, waits, LDS, instruction mix
set -e
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
O="$R/gpurun_out/pmc_attn"; mkdir -p "$O"
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $P -d "$O/p$i" -o run --output-format csv -- python3 "$R/tools/kbench.py" attn > "$O/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$O/p$i.log"; exit 1; }
done
python3 "$R/tools/pmc_summary.py" "$O" > "$O/summary.txt"
grep -i "attn\|kernel" "$O/summary.txt" | head -40
