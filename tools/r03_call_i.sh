#!/bin/bash
# Round-3 verification: full GPU suite (batch-32 parity reports in r03i/parity), the default
# bench line, rocprof kernel stats of the bench workload.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r03i
mkdir -p $O
PLD_REPORT_DIR=$O/parity timeout -k 10 900 python -u -m pytest -v -rf --timeout 900 --timeout-method thread -m gpu tests > $O/gputests.log 2>&1
rc=$?
echo "tests rc=$rc" >> $O/gputests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extra-configs --no-loss-parity > $R/$O/prof.log 2>&1 || exit 1
echo ok
