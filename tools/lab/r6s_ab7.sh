set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r6s
timeout -k 10 200 python -u tools/lab/epi_side_ab.py > gpurun_out/r6s/epi_side.jsonl 2>&1 || { cat gpurun_out/r6s/epi_side.jsonl; exit 1; }
cat gpurun_out/r6s/epi_side.jsonl
for q in 1 0 1; do
  OBST_G4W_QUEUE=$q timeout -k 10 300 python -u bench.py --config configs/ctx32_mixer.json --steps 5 --warmup 2 > gpurun_out/r6s/ctx32_q$q.log 2>&1 || exit 1
  echo "queue=$q $(tail -1 gpurun_out/r6s/ctx32_q$q.log | cut -c1-140)"
done
