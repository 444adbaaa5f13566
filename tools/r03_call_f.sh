#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r03f
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_kernels_gpu.py -k "conv" > $O/tests.log 2>&1 || exit 1
bash tools/ab_multi.sh pw "ab/pw_uniform/libpldepth_hip.so pldepth_amd/libpldepth_hip.so" "wgrad 32 56 56 240 240 144 3" "wgrad 32 112 112 144 144 32 3" "wgrad 32 224 224 32 0 32 3" "wgrad 32 112 112 64 0 16 3" > /dev/null 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-extra-configs --no-loss-parity > $O/bench.json 2> $O/bench.err || exit 1
