#!/bin/bash
# builds kernel-library variants of norm.hip (one .so per -D set) for tools/lab/norm_ctx32.py A/B runs
set -e
cd "$(dirname "$0")/../.."
HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -Wno-unused-result"
OTHERS=$(ls build/kernels/*.o | grep -v '/norm.o')
build() {
  tag=$1; shift
  /opt/rocm/bin/hipcc $HIPFLAGS "$@" -c csrc/kernels/norm.hip -o build/var/norm_$tag.o -Rpass-analysis=kernel-resource-usage 2> build/var/norm_$tag.ru
  /opt/rocm/bin/hipcc $HIPFLAGS -shared -o lab_so/k_$tag.so $OTHERS build/var/norm_$tag.o
  echo "$tag: $(grep -A3 'Function Name: .*norm_\(fwd\|bwd\)[a-z_0-9]*_kernelILi1E' build/var/norm_$tag.ru | grep -o 'VGPRs: [0-9]*' | tr '\n' ' ')"
}
for v in "$@"; do
  tag=${v%%:*}; flags=${v#*:}
  build $tag $flags &
done
wait
