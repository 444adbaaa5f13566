#!/bin/bash
# full GPU suite (incl. the batch-32 parity tests, reports in r03e/parity), then the ff_redweb
# weight-gradient overlap A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r03e
mkdir -p $O
PLD_REPORT_DIR=$O/parity timeout -k 10 1000 python -u -m pytest -v --timeout 900 --timeout-method thread -m gpu tests > $O/gputests.log 2>&1
echo "tests rc=$?" >> $O/gputests.log
for ov in 0 2; do
  PLD_OVERLAP_WGRAD=$ov timeout -k 10 200 python -u bench.py --model ff_redweb --no-cpu-baseline --no-extra-configs --no-loss-parity --tile-cache $O/tiles_rw.json > $O/rw_$ov.json 2>>$O/bench.err || exit 1
  python -c "import json;d=json.loads(open('$O/rw_$ov.json').read().strip().splitlines()[-1]);print('ff_redweb overlap=$ov', d['value'], d['ms_per_step'])" >> $O/ab.txt
done
bash tools/ab_multi.sh x3v "ab/base/libpldepth_hip.so pldepth_amd/libpldepth_hip.so ab/v_nosb/libpldepth_hip.so ab/v_pf3/libpldepth_hip.so" "wgrad 32 14 14 1280 0 672 3" "wgrad 32 28 28 1024 0 256 3" "wgrad 32 28 28 256 0 64 1" "wgrad 32 56 56 128 0 32 1" "dgrad 32 28 28 672 672 240 3" "fwd 32 28 28 672 672 240 3" "dgrad 32 14 14 1280 0 672 3" "fwd 32 28 28 672 0 112 1" "fwd 32 14 14 1152 0 192 1" > /dev/null 2>&1 || exit 1
