set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash tools/profile.sh r6s_ctx32_last --config configs/ctx32_mixer.json --steps 6 --warmup 3 > /dev/null || exit 1
head -16 gpurun_out/prof_r6s_ctx32_last/steps.md
