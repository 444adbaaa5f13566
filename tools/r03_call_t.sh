#!/bin/bash
# Whole-tile contiguous output stores in thin1x1 (output tile aliased over the input staging)
# and pgemm: kernel tests, thin micro A/B vs HEAD thin (ab/thin_old), ff_effnet bench on the
# current build, HEAD pgemm (ab/pg_old) and HEAD thin.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r03t
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_kernels_gpu.py -k "thin or pgemm or conv_fwd_dgrad" > $O/tests.log 2>&1 || exit 1
bash tools/ab_multi.sh thin2 "ab/thin_old/libpldepth_hip.so pldepth_amd/libpldepth_hip.so" "fwd 32 224 224 16 0 96 1" "fwd 32 112 112 24 0 144 1" "dgrad 32 112 112 144 0 24 1" "dgrad 32 224 224 96 0 16 1" > /dev/null 2>&1 || exit 1
cp gpurun_out/ab_thin2/ab.txt $O/ab_micro.txt
B="--no-cpu-baseline --no-loss-parity --no-extra-configs"
for lib in pldepth_amd ab/pg_old ab/thin_old pldepth_amd; do
  t=$(echo $lib | tr '/' '_')
  PLD_LIB_PATH=$lib/libpldepth_hip.so timeout -k 10 300 python -u bench.py $B >> $O/bench_$t.json 2>> $O/bench_$t.err || exit 1
done
echo ok
