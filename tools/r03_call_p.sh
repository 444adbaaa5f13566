#!/bin/bash
# Round-3 verification at HEAD: full GPU suite (batch-32 parity reports), the default bench line,
# rocprof kernel stats of the ff_effnet bench and of the ff_redweb bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r03p
mkdir -p $O
PLD_REPORT_DIR=$O/parity timeout -k 10 900 python -u -m pytest -v -rf --timeout 600 --timeout-method thread -m gpu tests > $O/gputests.log 2>&1
rc=$?
echo "tests rc=$rc" >> $O/gputests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extra-configs --no-loss-parity > $R/$O/prof.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_rw -o run --output-format csv -- python3 $R/bench.py --model ff_redweb --steps 6 --warmup 2 --no-cpu-baseline --no-extra-configs --no-loss-parity > $R/$O/prof_rw.log 2>&1 || exit 1
echo ok
