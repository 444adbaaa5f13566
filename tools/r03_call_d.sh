#!/bin/bash
# effnet bench A/B: decoder weight-gradient overlap mode x step-stream priority
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r03d
mkdir -p $O
for m in 0:0 1:0 2:0 2:1 1:1 0:1 0:0 2:0; do
  ov=${m%%:*}; pr=${m##*:}
  PLD_OVERLAP_WGRAD=$ov PLD_STREAM_PRIO=$pr timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-extra-configs --no-loss-parity --tile-cache $O/tiles.json > $O/b_$ov$pr.json 2>>$O/bench.err || exit 1
  python -c "import json;d=json.loads(open('$O/b_$ov$pr.json').read().strip().splitlines()[-1]);print('overlap=$ov prio=$pr', d['value'], d['ms_per_step'])" >> $O/ab.txt
done
