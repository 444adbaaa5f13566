#!/bin/bash
# GPU box: regenerate the persisted schedule table (bench.py --tune: cfg2 + cfg3 shapes, every
# schedule class incl. the tile streams), then the full GPU test suite on it
set -o pipefail
O=gpurun_out/r4h
mkdir -p $O
for v in bnhead new; do
  L=""; [ $v != new ] && L=ab/$v/libpldepth_hip.so
  PLD_LIB_PATH=$L timeout -k 10 300 python -u tools/bn_table.py --top 45 > $O/bn_$v.txt 2>&1 || { tail -20 $O/bn_$v.txt; exit 1; }
  tail -5 $O/bn_$v.txt
done
timeout -k 10 600 python -u bench.py --tune pldepth_amd/schedules/gfx950.json --no-cpu-baseline --no-loss-parity > $O/tune.json 2> $O/tune.err || { tail -20 $O/tune.err; exit 1; }
tail -c 600 $O/tune.json; echo
sha1sum pldepth_amd/schedules/gfx950.json
export PLD_REPORT_DIR=$O/parity
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
rc=$?
tail -5 $O/gputest.log
exit $rc
