#!/bin/bash
# A/B of the short-M bf16x3 tiles (GPU box): conv schedule kernel tests, conv_micro on the
# encoder's short-M 1x1 dgrad shapes, then the bench against ab/base (PLD_LIB_PATH). bash tools/ab_tiles.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
TAG=${1:-tiles}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "conv" > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/ab_micro.sh $TAG "dgrad 32 14 14 192 0 1152 1" "dgrad 32 14 14 1152 0 192 1" "dgrad 32 28 28 112 0 672 1" "dgrad 32 28 28 80 0 480 1" "dgrad 32 14 14 320 0 1280 1" "dgrad 32 14 14 672 0 192 1" "dgrad 32 28 28 672 0 112 1" > /dev/null || exit 1
B="--no-cpu-baseline --no-loss-parity"
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py $B >> $O/bench_new.json 2>> $O/bench_new.err || exit 1
  PLD_LIB_PATH=$R/ab/base/libpldepth_hip.so timeout -k 10 300 python -u bench.py $B >> $O/bench_base.json 2>> $O/bench_base.err || exit 1
done
echo ok
