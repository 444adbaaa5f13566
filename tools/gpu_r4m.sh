#!/bin/bash
# GPU box: full GPU suite (flip-aware ff_effnet gradient parity) + smoke
set -o pipefail
O=gpurun_out/r4m
mkdir -p $O
export PLD_REPORT_DIR=$O/parity
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 1000 --timeout-method thread > $O/gputest.log 2>&1
rc=$?
tail -4 $O/gputest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
exit $rc
