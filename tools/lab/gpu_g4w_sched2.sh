#!/bin/bash
# gemm4w schedule variants: timing over the step's shapes, in-kernel stamps and two PMC passes on d->2d
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/g4w
SKIP_CHECK=${SKIP_CHECK:-} timeout -k 10 300 $R/bin/g4w_sched 4 5 "" > $R/gpurun_out/g4w/time.txt 2>&1 || exit 1
grep "TF/s\| [1-9][0-9]*/[0-9]* bad" $R/gpurun_out/g4w/time.txt
STAMPS=1 SKIP_CHECK=1 timeout -k 10 120 $R/bin/g4w_sched 1 2 "fwd d->2d" > $R/gpurun_out/g4w/stamps.txt 2>&1 || exit 1
grep stamps $R/gpurun_out/g4w/stamps.txt
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  G4W_ONLY=1,2,3 SKIP_CHECK=1 timeout -s KILL 90 rocprofv3 --pmc $P -d $R/gpurun_out/g4w/p$i -o run --output-format csv -- $R/bin/g4w_sched 1 2 "fwd d->2d" > $R/gpurun_out/g4w/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -3 $R/gpurun_out/g4w/p$i.log; exit 1; }
done
python3 $R/tools/pmc_summary.py $R/gpurun_out/g4w > $R/gpurun_out/g4w/pmc.txt && cat $R/gpurun_out/g4w/pmc.txt
cd $R && timeout -k 10 300 python -u tools/kbench.py mixer > $R/gpurun_out/g4w/mixer.txt 2>&1 && cat $R/gpurun_out/g4w/mixer.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "gemm or mixer" > $R/gpurun_out/g4w/tests.txt 2>&1; tail -5 $R/gpurun_out/g4w/tests.txt
