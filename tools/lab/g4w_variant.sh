#!/bin/bash
# builds a kernel-library variant with the gemm4w translation units compiled under extra -D flags
# usage: tools/lab/g4w_variant.sh <tag> <flags...>   -> lab_so/k_<tag>.so
set -e
cd "$(dirname "$0")/../.."
tag=$1; shift
HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -Wno-unused-result"
mkdir -p build/var/g4w_$tag lab_so
for f in csrc/kernels/gemm4w*.hip csrc/kernels/gemm.hip; do
  b=$(basename $f .hip)
  /opt/rocm/bin/hipcc $HIPFLAGS "$@" -c $f -o build/var/g4w_$tag/$b.o &
done
wait
OTHERS=$(ls build/kernels/*.o | grep -v '/gemm4w\|/gemm.o')
/opt/rocm/bin/hipcc $HIPFLAGS -shared -o lab_so/k_$tag.so $OTHERS build/var/g4w_$tag/*.o
echo built lab_so/k_$tag.so
