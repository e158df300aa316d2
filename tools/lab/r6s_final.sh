set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --config configs/ctx32_mixer.json --steps 10 --warmup 3 > gpurun_out/ctx32_final.log 2>&1 || { tail -20 gpurun_out/ctx32_final.log; exit 1; }
tail -1 gpurun_out/ctx32_final.log | cut -c1-160
PROFILE_TAG=r6s_final2 bash tools/gpu_final.sh
