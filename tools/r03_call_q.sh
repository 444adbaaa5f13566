#!/bin/bash
# PMC HBM traffic of one eager ff_effnet step at HEAD (FETCH_SIZE / WRITE_SIZE passes), then the
# conv2-stage exactness experiment (which of the stage's convs need exact fp32 in the forward).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r03q
mkdir -p $O
bash tools/prof_step_pmc.sh ff_effnet > $O/pmc.log 2>&1 || exit 1
cd $R
timeout -k 10 900 python -u tools/exp_redweb_policy2.py > $O/policy2.log 2>&1 || exit 1
echo ok
