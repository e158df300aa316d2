set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r6s
for v in tree nt1 nt2 nt3; do
  if [ $v = tree ]; then unset OBST_KERNELS; else export OBST_KERNELS=$PWD/lab_so/k_$v.so; fi
  timeout -k 10 120 python -u tools/lab/norm_ctx32.py --tag $v >> gpurun_out/r6s/norm_ab5.jsonl 2> gpurun_out/r6s/norm_ab5_$v.err || exit 1
done
cat gpurun_out/r6s/norm_ab5.jsonl
for v in tree zcpnt tree; do
  if [ $v = tree ]; then unset OBST_KERNELS; else export OBST_KERNELS=$PWD/lab_so/k_$v.so; fi
  timeout -k 10 300 python -u bench.py --config configs/ctx32_mixer.json --steps 5 --warmup 2 > gpurun_out/r6s/ctx32_ab5_$v.log 2>&1 || exit 1
  echo "$v $(tail -1 gpurun_out/r6s/ctx32_ab5_$v.log | cut -c1-140)"
done
