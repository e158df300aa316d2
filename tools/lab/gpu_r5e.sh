#!/bin/bash
# Round-5 profiles: headline step profile, ctx32_mixer step profile, kernel gate floors
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
bash tools/profile.sh r5f --steps 6 --warmup 3 || exit 1
bash tools/profile.sh r5ctx --config configs/ctx32_mixer.json --steps 4 --warmup 2 || exit 1
timeout -k 10 600 python -u tools/kbench.py all --write-floors gpurun_out/kbench_floor_new.json > gpurun_out/kbench.log 2>&1 || { tail -20 gpurun_out/kbench.log; exit 1; }
tail -5 gpurun_out/kbench.log
