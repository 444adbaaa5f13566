#!/bin/bash
# Build an A/B copy of libpldepth_hip.so with ONE source file taken from a git revision:
#   bash tools/ab_lib.sh REV pldepth_amd/csrc/FILE.hip OUT_DIR
# (the other objects come from the current in-tree build). Load it with PLD_LIB_PATH=OUT_DIR/...
set -e
REV=$1; SRC=$2; OUT=$3
mkdir -p $OUT
git show $REV:$SRC > $OUT/$(basename $SRC)
cp pldepth_amd/csrc/*.h $OUT/
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Wno-unused-function \
  -Wno-unused-variable -munsafe-fp-atomics -Iinclude -c $OUT/$(basename $SRC) -o $OUT/ab.o
OBJS=$(ls build/hip/*.o)
OBJS=$(echo "$OBJS" | grep -v "/$(basename $SRC).o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libpldepth_hip.so $OUT/ab.o $OBJS
echo $OUT/libpldepth_hip.so
