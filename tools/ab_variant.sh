#!/bin/bash
# Build an A/B copy of libpldepth_hip.so with conv_x3.hip compiled under extra -D flags:
#   bash tools/ab_variant.sh OUT_DIR -DX3_FOO [-DX3_BAR ...]
set -e
OUT=$1; shift
mkdir -p $OUT
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Wno-unused-function \
  -Wno-unused-variable -munsafe-fp-atomics -Iinclude "$@" -c pldepth_amd/csrc/conv_x3.hip -o $OUT/ab.o
OBJS=$(ls build/hip/*.o | grep -v "/conv_x3.hip.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libpldepth_hip.so $OUT/ab.o $OBJS
echo $OUT/libpldepth_hip.so
