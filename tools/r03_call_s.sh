#!/bin/bash
# thin 1x1 kernel storing its whole [64][N] tile as one contiguous run vs HEAD (ab/thin_old):
# kernel tests, per-shape micro A/B, ff_effnet bench on both.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r03s
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_kernels_gpu.py -k "thin or conv_fwd_dgrad or every_schedule" > $O/tests.log 2>&1 || exit 1
bash tools/ab_multi.sh thin "ab/thin_old/libpldepth_hip.so pldepth_amd/libpldepth_hip.so" "fwd 32 224 224 16 0 96 1" "fwd 32 112 112 24 0 144 1" "dgrad 32 112 112 144 0 24 1" "dgrad 32 224 224 96 0 16 1" "fwd 32 56 56 40 0 96 1" > /dev/null 2>&1 || exit 1
cp gpurun_out/ab_thin/ab.txt $O/ab_micro.txt
B="--no-cpu-baseline --no-loss-parity --no-extra-configs"
timeout -k 10 300 python -u bench.py $B > $O/bench_eff.json 2> $O/bench_eff.err || exit 1
PLD_LIB_PATH=ab/thin_old/libpldepth_hip.so timeout -k 10 300 python -u bench.py $B > $O/bench_eff_old.json 2> $O/bench_eff_old.err || exit 1
timeout -k 10 300 python -u bench.py $B > $O/bench_eff2.json 2> $O/bench_eff2.err || exit 1
echo ok
