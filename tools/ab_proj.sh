#!/bin/bash
# ff_redweb projection-shortcut overlap A/B (GPU box): PLD_OVERLAP_PROJ=1 vs 0, cfg3 bench, 3 reps.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/${1:-proj}
mkdir -p $O
B="--model ff_redweb --no-cpu-baseline --no-loss-parity --no-extra-configs"
for rep in 1 2 3; do
  PLD_OVERLAP_PROJ=1 timeout -k 10 300 python -u bench.py $B >> $O/p1.json 2>> $O/err.log || exit 1
  PLD_OVERLAP_PROJ=0 timeout -k 10 300 python -u bench.py $B >> $O/p0.json 2>> $O/err.log || exit 1
done
echo ok
