#!/bin/bash
# PLD_DW_BNB A/B at HEAD (the expand BN's backward reductions in the depthwise dgrad epilogue vs
# the separate reduction pass), alternating, two lines each.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r03u
mkdir -p $O
B="--no-cpu-baseline --no-loss-parity --no-extra-configs"
for rep in 1 2; do
  for m in 0 1; do
    PLD_DW_BNB=$m timeout -k 10 300 python -u bench.py $B >> $O/bench_dwbnb$m.json 2>> $O/bench_dwbnb$m.err || exit 1
  done
done
echo ok
