#!/bin/bash
# BN add-backward dz pass + forward-only exact conv2 stage (ff_redweb): kernel tests, the
# bench-policy parity test of ff_redweb, cfg3 bench line (default env and exact backward A/B),
# BN table.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r03l
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_kernels_gpu.py -k "bn" > $O/tests.log 2>&1 || exit 1
PLD_REPORT_DIR=$O/parity timeout -k 10 600 python -u -m pytest -x -v --timeout 600 --timeout-method thread "tests/test_configs_gpu.py::test_batch32_bench_policy[ff_redweb]" > $O/policy.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --model ff_redweb --no-cpu-baseline --no-loss-parity --no-extra-configs > $O/bench_rw.json 2> $O/bench_rw.err || exit 1
PLD_REDWEB_EXACT_BWD=1 timeout -k 10 300 python -u bench.py --model ff_redweb --no-cpu-baseline --no-loss-parity --no-extra-configs > $O/bench_rw_exactbwd.json 2> $O/bench_rw_exactbwd.err || exit 1
timeout -k 10 200 python -u tools/bn_table.py --model ff_redweb --top 30 > $O/bn_redweb.txt 2>&1 || exit 1
echo ok
