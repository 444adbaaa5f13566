#!/bin/bash
# GPU box: re-tune the schedule table at HEAD (written under gpurun_out, copied into the tree
# copy for the tests), the full GPU suite on it, smoke
set -o pipefail
O=gpurun_out/r4t
mkdir -p $O
timeout -k 10 600 python -u bench.py --tune $O/gfx950.json --no-cpu-baseline --no-loss-parity > $O/tune.json 2> $O/tune.err || { tail -20 $O/tune.err; exit 1; }
cp $O/gfx950.json pldepth_amd/schedules/gfx950.json && sha1sum pldepth_amd/schedules/gfx950.json
export PLD_REPORT_DIR=$O/parity
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 1000 --timeout-method thread > $O/gputest.log 2>&1
rc=$?
tail -4 $O/gputest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
exit $rc
