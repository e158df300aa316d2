set -o pipefail
mkdir -p gpurun_out
for kg in 2; do
  OBST_ATTN_DKV_KG=$kg timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k attention > gpurun_out/kg_test$kg.log 2>&1 || { echo "test kg=$kg failed"; tail -30 gpurun_out/kg_test$kg.log; exit 1; }
  tail -1 gpurun_out/kg_test$kg.log
done
for kg in 1 2 1 2; do
  echo "KG=$kg"; OBST_ATTN_DKV_KG=$kg B=64 timeout -k 10 120 python -u tools/lab/bench_attn.py 2>&1 | grep attn || exit 1
done
