#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r03g
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_kernels_gpu.py -k "conv" > $O/tests.log 2>&1 || exit 1
bash tools/ab_multi.sh mc "ab/mc_uniform/libpldepth_hip.so pldepth_amd/libpldepth_hip.so" "fwd 32 56 56 240 240 144 3" "dgrad 32 56 56 240 240 144 3" "fwd 32 112 112 144 144 32 3" "dgrad 32 112 112 144 144 32 3" "fwd 32 56 56 128 0 128 3" > /dev/null 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-loss-parity > $O/bench.json 2> $O/bench.err || exit 1
