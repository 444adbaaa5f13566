#!/bin/bash
# LDS-tiled stride-1 depthwise dgrad (dw tile kernel, DG form): kernel tests, model tests,
# bench A/B against the HEAD dwtile.hip + dwse.hip (ab/base).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r03y
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_kernels_gpu.py -k "dwconv or se_" > $O/tests.log 2>&1 || exit 1
PLD_REPORT_DIR=$O/parity timeout -k 10 900 python -u -m pytest -v --timeout 600 --timeout-method thread tests/test_model_gpu.py "tests/test_configs_gpu.py::test_batch32_bench_policy[ff_effnet]" tests/test_configs_gpu.py::test_effnet_448_bf16x3_gradients > $O/model_tests.log 2>&1
rc=$?; echo "rc=$rc" >> $O/model_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
B="--no-cpu-baseline --no-loss-parity --no-extra-configs"
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py $B >> $O/bench_new.json 2>> $O/bench_new.err || exit 1
  PLD_LIB_PATH=$R/ab/base/libpldepth_hip.so timeout -k 10 300 python -u bench.py $B >> $O/bench_base.json 2>> $O/bench_base.err || exit 1
done
echo ok
