#!/bin/bash
# BN add-backward dz pass, forward-only exact conv2 stage, bf16x3 conv input prologue (ff_redweb
# encoder conv2/conv3 read the pre-BN tensors through BN + ReLU): kernel tests, the ff_redweb
# bench-policy parity test, cfg3 bench A/B (prologue on/off, exact backward), BN table.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r03m
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "bn or prologue or conv_fwd_dgrad" > $O/tests.log 2>&1 || exit 1
PLD_REPORT_DIR=$O/parity timeout -k 10 600 python -u -m pytest -x -v --timeout 600 --timeout-method thread "tests/test_configs_gpu.py::test_batch32_bench_policy[ff_redweb]" tests/test_redweb_gpu.py > $O/policy.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --model ff_redweb --no-cpu-baseline --no-loss-parity --no-extra-configs > $O/bench_rw.json 2> $O/bench_rw.err || exit 1
PLD_BN_PROLOGUE=0 timeout -k 10 300 python -u bench.py --model ff_redweb --no-cpu-baseline --no-loss-parity --no-extra-configs > $O/bench_rw_nopro.json 2> $O/bench_rw_nopro.err || exit 1
PLD_REDWEB_EXACT_BWD=1 timeout -k 10 300 python -u bench.py --model ff_redweb --no-cpu-baseline --no-loss-parity --no-extra-configs > $O/bench_rw_exactbwd.json 2> $O/bench_rw_exactbwd.err || exit 1
timeout -k 10 200 python -u tools/bn_table.py --model ff_redweb --top 30 > $O/bn_redweb.txt 2>&1 || exit 1
timeout -k 10 200 python -u tools/conv_table.py --model ff_effnet --math auto --top 60 > $O/conv_table_effnet.txt 2>&1 || exit 1
echo ok
