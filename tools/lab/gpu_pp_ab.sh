set -o pipefail
mkdir -p gpurun_out
OBST_GEMM_LT=0 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "gemm or mixer" > gpurun_out/pp_t.log 2>&1 || { tail -30 gpurun_out/pp_t.log; exit 1; }
tail -1 gpurun_out/pp_t.log
for v in 0 1; do echo "OBST_GEMM_PP=$v"; OBST_GEMM_PP=$v timeout -k 10 200 python -u tools/lab/bench_ph_layouts.py || exit 1; done
for v in 0 1 0 1; do echo "ctx32 OBST_GEMM_PP=$v: $(OBST_GEMM_PP=$v timeout -k 10 300 python bench.py --config configs/ctx32_mixer.json --steps 6 --warmup 3 --batch-per-gpu 32 2>/dev/null | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" || exit 1; done
