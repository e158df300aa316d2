#!/bin/bash
# kernel-library variants differing only in the gemm4w stream-update instantiation's options: ab/zcp_<opt>.so
set -e
cd "$(dirname "$0")/../.."
make -s >/dev/null
mkdir -p ab build/var
OBJS=$(ls build/kernels/*.o | grep -v -e gemm4w_00.o -e gemm4w_01.o)
for opt in "$@"; do
  for tu in 00 01; do
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -Wno-unused-result \
      -DG4W_ZCP_OPT=$opt -c csrc/kernels/gemm4w_$tu.hip -o build/var/g4w_${tu}_zcp$opt.o &
  done
  wait
  /opt/rocm/bin/hipcc -O3 -fPIC --offload-arch=gfx950 -shared -o ab/zcp_$opt.so $OBJS build/var/g4w_00_zcp$opt.o build/var/g4w_01_zcp$opt.o
done
ls -la ab/zcp_*.so
