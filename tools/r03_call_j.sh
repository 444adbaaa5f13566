#!/bin/bash
# conv tests (the double-buffered 64-cout patch WGRAD) and its A/B against the single-stage one
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r03j
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_kernels_gpu.py -k "conv" > $O/tests.log 2>&1 || exit 1
bash tools/ab_multi.sh pw64 "ab/pw64_single/libpldepth_hip.so pldepth_amd/libpldepth_hip.so" "wgrad 32 28 28 672 672 240 3" "wgrad 32 56 56 240 240 112 3" "wgrad 32 14 14 1280 0 672 3" > /dev/null 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-loss-parity --no-extra-configs > $O/bench.json 2> $O/bench.err || exit 1
