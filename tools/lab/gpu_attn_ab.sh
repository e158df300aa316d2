# attention kernel A/B over one environment variable: VAR=name VALS="a b a b" (tests + bench_attn per value)
set -o pipefail
mkdir -p gpurun_out
for v in $VALS; do
  env $VAR=$v timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k attention > gpurun_out/attn_ab_test.log 2>&1 || { echo "test $VAR=$v failed"; tail -30 gpurun_out/attn_ab_test.log; exit 1; }
  echo "$VAR=$v: $(tail -1 gpurun_out/attn_ab_test.log)"; env $VAR=$v B=64 timeout -k 10 120 python -u tools/lab/bench_attn.py 2>&1 | grep attn || exit 1
done
