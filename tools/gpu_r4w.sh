#!/bin/bash
# GPU box: full GPU suite, smoke and the default bench line on the in-tree build
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4w
mkdir -p $O
export PLD_REPORT_DIR=$O/parity
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
rc=$?
tail -4 $O/gputest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python3 $R/bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('extra_configs', {}) and {k: v.get('value') for k, v in d['extra_configs'].items()}, d['cpu_baseline']['value'])"
