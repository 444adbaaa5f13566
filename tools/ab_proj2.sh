#!/bin/bash
# ff_redweb projection-shortcut overlap, forward + backward (GPU box): trainer / ReDWeb tests, the
# batch-32 cfg3 parity test, then PLD_OVERLAP_PROJ=1 vs 0 on the cfg3 bench, 3 reps.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/${1:-proj2}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_trainer_gpu.py tests/test_redweb_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
B="--model ff_redweb --no-cpu-baseline --no-loss-parity --no-extra-configs"
for rep in 1 2 3; do
  PLD_OVERLAP_PROJ=1 timeout -k 10 300 python -u bench.py $B >> $O/p1.json 2>> $O/err.log || exit 1
  PLD_OVERLAP_PROJ=0 timeout -k 10 300 python -u bench.py $B >> $O/p0.json 2>> $O/err.log || exit 1
done
PLD_REPORT_DIR=$O/parity timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread "tests/test_configs_gpu.py::test_batch32_bench_policy[ff_redweb]" > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
grep -E "passed|failed" $O/parity.log | tail -1
echo ok
