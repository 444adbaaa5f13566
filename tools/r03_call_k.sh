#!/bin/bash
# Round-3 re-entry check at HEAD: full GPU suite, the default bench line, BN call tables of
# both models, the ff_redweb conv table under auto.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r03k
mkdir -p $O
PLD_REPORT_DIR=$O/parity timeout -k 10 900 python -u -m pytest -v -rf --timeout 300 --timeout-method thread -m gpu tests > $O/gputests.log 2>&1
rc=$?
echo "tests rc=$rc" >> $O/gputests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 200 python -u tools/bn_table.py --model ff_redweb --top 60 > $O/bn_redweb.txt 2>&1 || exit 1
timeout -k 10 200 python -u tools/bn_table.py --model ff_effnet --top 40 > $O/bn_effnet.txt 2>&1 || exit 1
timeout -k 10 200 python -u tools/conv_table.py --model ff_redweb --math auto --top 80 > $O/conv_table_redweb.txt 2>&1 || exit 1
echo ok
