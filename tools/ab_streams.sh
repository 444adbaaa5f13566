#!/bin/bash
# Filter refresh over several streams (PLD_REFRESH_STREAMS) and the ff_redweb projection-shortcut
# overlap (with PLD_OVERLAP_FFL) — GPU box: trainer / model tests, then bench A/B, two reps each.
# bash tools/ab_streams.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
TAG=${1:-streams}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_trainer_gpu.py tests/test_redweb_gpu.py tests/test_model_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
B="--no-cpu-baseline --no-loss-parity --no-extra-configs"
for rep in 1 2; do
  PLD_REFRESH_STREAMS=4 timeout -k 10 300 python -u bench.py $B >> $O/eff_r4.json 2>> $O/err.log || exit 1
  PLD_REFRESH_STREAMS=1 timeout -k 10 300 python -u bench.py $B >> $O/eff_r1.json 2>> $O/err.log || exit 1
  PLD_REFRESH_STREAMS=4 timeout -k 10 300 python -u bench.py --model ff_redweb $B >> $O/rw_r4.json 2>> $O/err.log || exit 1
  PLD_REFRESH_STREAMS=1 timeout -k 10 300 python -u bench.py --model ff_redweb $B >> $O/rw_r1.json 2>> $O/err.log || exit 1
done
echo ok
