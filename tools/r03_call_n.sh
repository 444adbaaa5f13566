#!/bin/bash
# ff_redweb conv input prologue A/B: cfg3 bench per PLD_BN_PROLOGUE mode (0 off, 1 conv2+conv3,
# 2 conv3 only, 3 conv2 only) and per-conv tables with it on / off; ff_effnet default bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r03n
mkdir -p $O
for m in 0 1 2 3; do
  PLD_BN_PROLOGUE=$m timeout -k 10 300 python -u bench.py --model ff_redweb --no-cpu-baseline --no-loss-parity --no-extra-configs > $O/bench_rw_p$m.json 2> $O/bench_rw_p$m.err || exit 1
done
PLD_BN_PROLOGUE=1 timeout -k 10 200 python -u tools/conv_table.py --model ff_redweb --math auto --top 200 > $O/conv_table_rw_p1.txt 2>&1 || exit 1
PLD_BN_PROLOGUE=0 timeout -k 10 200 python -u tools/conv_table.py --model ff_redweb --math auto --top 200 > $O/conv_table_rw_p0.txt 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-loss-parity --no-extra-configs > $O/bench_eff.json 2> $O/bench_eff.err || exit 1
echo ok
