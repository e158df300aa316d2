#!/bin/bash
# Device assembly of one kernel source for gfx950 (inspect schedules / register counts): tools/asm_kernel.sh src.hip out.s
set -e
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 --cuda-device-only -S -Wno-unused-result "${@:3}" "$1" -o "$2"
