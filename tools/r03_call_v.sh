#!/bin/bash
# expand-BN backward with expand_pre recomputed from the block input (PLD_EXPAND_RC): kernel
# tests, ff_effnet whole-model tests, bench A/B (alternating, two lines each).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r03v
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_kernels_gpu.py -k "recompute or pgemm or thin or dwconv_dgrad_bn" > $O/tests.log 2>&1 || exit 1
PLD_REPORT_DIR=$O/parity timeout -k 10 900 python -u -m pytest -v --timeout 600 --timeout-method thread tests/test_model_gpu.py "tests/test_configs_gpu.py::test_batch32_bench_policy[ff_effnet]" tests/test_configs_gpu.py::test_effnet_448_bf16x3_gradients > $O/model_tests.log 2>&1
rc=$?; echo "rc=$rc" >> $O/model_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
B="--no-cpu-baseline --no-loss-parity --no-extra-configs"
for rep in 1 2; do
  for m in 1 0; do
    PLD_EXPAND_RC=$m timeout -k 10 300 python -u bench.py $B >> $O/bench_rc$m.json 2>> $O/bench_rc$m.err || exit 1
  done
done
echo ok
