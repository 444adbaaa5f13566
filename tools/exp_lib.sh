#!/bin/bash
# Timing-only variant of libpldepth_hip.so: conv_x3_grid.hip recompiled with extra flags
# (e.g. -DX3_EXP_NOB=1), the other objects from the in-tree build. Load it with PLD_LIB_PATH.
#   bash tools/exp_lib.sh OUT_DIR -DFLAG=1 ...
set -e
OUT=$1; shift
mkdir -p $OUT
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Wno-unused-function \
  -Wno-unused-variable -munsafe-fp-atomics -Iinclude -Ipldepth_amd/csrc "$@" \
  -c pldepth_amd/csrc/conv_x3_grid.hip -o $OUT/grid.o
OBJS=$(ls build/hip/*.o | grep -v "/conv_x3_grid.hip.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libpldepth_hip.so $OUT/grid.o $OBJS
echo $OUT/libpldepth_hip.so
