#!/bin/bash
# GPU box: full GPU test suite, the default bench line (cpu_baseline, loss parity, extra configs)
# and a rocprofv3 kernel trace of the graph-replayed bench steps with per-step kernel stats.
# bash tools/gpu_verify.sh TAG [--no-tests]
set -o pipefail
TAG=${1:-verify}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
TEST_RC=0
# progress marker for the GPU pool's silence watchdog (a parity test's fp64 oracle runs
# several minutes without printing); every step below keeps its own time limit
(while sleep 45; do date >> $O/heartbeat.txt; done) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
if [ "$2" != "--no-tests" ]; then
  export PLD_REPORT_DIR=$O/parity
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
  TEST_RC=$?
  tail -3 $O/gputest.log
  # a test failure (1) still lets the bench / trace run; anything else (a crash, a time limit)
  # ends the call; either way the script's exit status reports it
  if [ $TEST_RC -ne 0 ] && [ $TEST_RC -ne 1 ]; then exit $TEST_RC; fi
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python3 $R/bench.py > $O/bench.json 2> $O/bench.err || exit 1
tail -c 400 $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-loss-parity --no-extra-configs > $O/trace.log 2>&1 || exit 1
DB=$(ls $O/trace/*/run_results.db 2>/dev/null | head -1)
[ -z "$DB" ] && DB=$(ls $O/trace/run_results.db 2>/dev/null | head -1)
python3 $R/tools/kstats.py $DB --marker adam_amsgrad_dev_kernel --steps 10 --skip 1 --csv $O/kernel_stats.csv --top 70 > $O/kstats.txt || exit 1
rm -rf $O/trace
head -3 $O/kstats.txt
echo done
exit $TEST_RC
