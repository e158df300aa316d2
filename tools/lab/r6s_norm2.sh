set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r6s
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "norm" --timeout 120 --timeout-method thread > gpurun_out/r6s/norm4_tests.log 2>&1 || { tail -30 gpurun_out/r6s/norm2_tests.log; exit 1; }
tail -1 gpurun_out/r6s/norm4_tests.log
for v in tree nt1 nt2 nt3 tree; do
  if [ $v = tree ]; then unset OBST_KERNELS; else export OBST_KERNELS=$PWD/lab_so/k_$v.so; fi
  timeout -k 10 120 python -u tools/lab/norm_ctx32.py --tag $v$([ -e gpurun_out/r6s/seen4_$v ] && echo _2; touch gpurun_out/r6s/seen4_$v) >> gpurun_out/r6s/norm_ab4.jsonl 2> gpurun_out/r6s/norm_ab4_$v.err || exit 1
done
unset OBST_KERNELS
cat gpurun_out/r6s/norm_ab4.jsonl
timeout -k 10 300 python -u bench.py --config configs/ctx32_mixer.json --steps 5 --warmup 2 > gpurun_out/r6s/ctx32_4.log 2>&1 && tail -1 gpurun_out/r6s/ctx32_4.log | cut -c1-200
