#!/bin/bash
# ff_redweb FFL left-branch overlap (GPU box): ReDWeb model / trainer tests, then cfg3 bench with
# PLD_OVERLAP_FFL=1 vs 0 (two reps each). bash tools/ab_ffl.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
TAG=${1:-ffl}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_trainer_gpu.py tests/test_redweb_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
B="--model ff_redweb --no-cpu-baseline --no-loss-parity --no-extra-configs"
for rep in 1 2; do
  PLD_OVERLAP_FFL=1 timeout -k 10 300 python -u bench.py $B >> $O/bench_on.json 2>> $O/bench_on.err || exit 1
  PLD_OVERLAP_FFL=0 timeout -k 10 300 python -u bench.py $B >> $O/bench_off.json 2>> $O/bench_off.err || exit 1
done
PLD_REPORT_DIR=$O/parity timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread "tests/test_configs_gpu.py::test_batch32_bench_policy[ff_redweb]" > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
grep -E "passed|failed" $O/parity.log | tail -1
echo ok
