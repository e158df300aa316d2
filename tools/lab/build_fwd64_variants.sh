#!/bin/bash
# Build kernel-library variants that differ only in attn_fwd64.o's -D flags: ab/f64_<name>.so
# usage: tools/lab/build_fwd64_variants.sh "name:-DFOO=1 -DBAR=2" ...
set -e
cd "$(dirname "$0")/../.."
make -s >/dev/null
mkdir -p ab build/var
OBJS=$(ls build/kernels/*.o | grep -v attn_fwd64.o)
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -Wno-unused-result -fno-slp-vectorize $flags \
    -c csrc/kernels/attn_fwd64.hip -o build/var/f64_$name.o -Rpass-analysis=kernel-resource-usage 2> build/var/f64_$name.rpt
  grep -A9 "attn_fwd64_kernel" build/var/f64_$name.rpt | grep -E "VGPRs:|AGPRs|Spill: [1-9]" | sed "s/^.*remark: *//" | tr '\n' ' '; echo " <- $name"
  /opt/rocm/bin/hipcc -O3 -fPIC --offload-arch=gfx950 -shared -o ab/f64_$name.so $OBJS build/var/f64_$name.o
done
