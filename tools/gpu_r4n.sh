#!/bin/bash
# GPU box: the ReDWeb batch-32 flip-aware parity test, the default bench line (reads the r04
# profiles: traffic, MFMA busy, step bytes), SQ counters of the dominant kernel's largest launch
set -o pipefail
O=gpurun_out/r4n
mkdir -p $O
PLD_REPORT_DIR=$O/parity timeout -k 10 1100 python -u -m pytest tests/test_configs_gpu.py -q -x -k "batch32 and redweb" --timeout 1050 --timeout-method thread > $O/rw.log 2>&1
rc=$?
tail -3 $O/rw.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python3 $GRAFT_REPO_ROOT/bench.py > $GRAFT_REPO_ROOT/$O/bench.json 2> $GRAFT_REPO_ROOT/$O/bench.err || exit 1
tail -c 300 $GRAFT_REPO_ROOT/$O/bench.json
cd $GRAFT_REPO_ROOT
bash tools/gpu_pmc1.sh r4n/pmc_dec0fwd --mode fwd --n 32 --h 14 --w 14 --c1 1280 --k 3 --cout 672 --sched 35 > $O/pmc_dec0fwd.txt 2>&1 || { cat $O/pmc_dec0fwd.txt; exit 1; }
head -2 $O/pmc_dec0fwd.txt
bash tools/gpu_pmc1.sh r4n/pmc_dec1dgrad --mode dgrad --n 32 --h 28 --w 28 --c1 672 --c2 672 --k 3 --cout 240 --sched 16 > $O/pmc_dec1dgrad.txt 2>&1 || { cat $O/pmc_dec1dgrad.txt; exit 1; }
head -2 $O/pmc_dec1dgrad.txt
exit $rc
