set -o pipefail
mkdir -p gpurun_out
for e in ""; do
  SKIP_CHECK=1 STAMPS=1 timeout -k 10 120 bin/gemm_bench$e 2 3 "131072x4096x2048" > gpurun_out/exp$e.log 2>&1 || { echo "fail $e"; tail -5 gpurun_out/exp$e.log; exit 1; }
  echo "== variant $e"; grep "stamps\|TF/s" gpurun_out/exp$e.log
done
