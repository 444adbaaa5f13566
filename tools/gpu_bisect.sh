#!/bin/bash
# GPU box: the cfg1 whole-step gradient test and the 64^2 forward-activation test in complete
# copies of earlier revisions (ab/bisect/REV: sources + their own built library), to find the
# commit that moved the gradient parity (global rel-L2 0.0073 at r03 -> 0.0116)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/bisect
mkdir -p $O
for r in "$@"; do
  if [ "$r" = HEAD ]; then cd $GRAFT_REPO_ROOT; else cd $GRAFT_REPO_ROOT/ab/bisect/$r || exit 1; fi
  PLD_REPORT_DIR=$O/$r timeout -k 10 400 python -u -m pytest tests/test_configs_gpu.py::test_cfg1_trainer_step_224 tests/test_model_gpu.py::test_forward_activations -q --timeout 300 --timeout-method thread > $O/$r.log 2>&1
  echo "$r rc=$?"; tail -2 $O/$r.log
  python3 -c "import json; d=json.load(open('$O/$r/parity_cfg1_224.json')); print('$r', d['global'])" 2>/dev/null
done
