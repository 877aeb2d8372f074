#!/bin/bash
# Build an alternative kernel library for A/B runs: tools/build_variant.sh NAME [hipcc flags...]
# -> textblaster_amd/libtbhip_NAME.so ; select it with TB_HIP_LIB=<path>. Only kernels.hip takes the
# flags; the runtime layer and the HTML kernels are linked from the default build (build/hip/).
set -e
cd "$(dirname "$0")/.."
name=$1; shift
mkdir -p build/variants
python3 -c "from textblaster_amd import native; native.build_hip()" > /dev/null
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fno-gpu-rdc -fconstexpr-steps=200000000 "$@" -c csrc/hip/kernels.hip \
  -o build/variants/kernels_$name.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o textblaster_amd/libtbhip_$name.so build/variants/kernels_$name.o \
  $(ls build/hip/*.o | grep -v kernels.hip.o)
echo textblaster_amd/libtbhip_$name.so
