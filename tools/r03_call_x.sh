#!/bin/bash
# Split A/B of call w (reduce grid vs SE squeeze split), the depthwise tile-loop kernel
# (2 / 3 workgroups per CU), kernel tests of the in-tree build, rocprof stats new vs base.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r03x
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_kernels_gpu.py -k "dwconv or se_" > $O/tests.log 2>&1 || exit 1
B="--no-cpu-baseline --no-loss-parity --no-extra-configs"
for rep in 1 2; do
  for v in base bn_only se_only dw2 dw3; do
    PLD_LIB_PATH=$R/ab/$v/libpldepth_hip.so timeout -k 10 300 python -u bench.py $B >> $O/bench_$v.json 2>> $O/bench_$v.err || exit 1
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_new -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 $B > $R/$O/prof_new.log 2>&1 || exit 1
PLD_LIB_PATH=$R/ab/base/libpldepth_hip.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_base -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 $B > $R/$O/prof_base.log 2>&1 || exit 1
echo ok
