#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/r03c
for m in ff_effnet:0 ff_effnet:1 ff_effnet:0 ff_effnet:1 ff_redweb:0 ff_redweb:1; do
  model=${m%%:*}; ov=${m##*:}
  PLD_OVERLAP_WGRAD=$ov timeout -k 10 300 python -u bench.py --model $model --no-cpu-baseline --no-extra-configs --no-loss-parity --tile-cache gpurun_out/r03c/tiles_$model.json > gpurun_out/r03c/bench_${model}_ov$ov.json 2>>gpurun_out/r03c/bench.err || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/r03c/bench_${model}_ov$ov.json').read().strip().splitlines()[-1]);print('$model overlap=$ov', d['value'], d['ms_per_step'])" >> gpurun_out/r03c/overlap_ab.txt
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_trainer_gpu.py tests/test_model_gpu.py tests/test_redweb_gpu.py > gpurun_out/r03c/tests.log 2>&1 || exit 1
./tools/exp_x3_flags.sh || exit 1
