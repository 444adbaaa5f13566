#!/bin/bash
# Consumer-side bf16 split of the im2col A operand (X3_CSPLIT=1, in-tree) vs the producer split
# (ab/cs0): conv kernel tests, conv micro A/B on the dominant shapes, both benches, the ff_redweb
# conv input prologue modes on the new build.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r03o
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "conv or pgemm" > $O/tests.log 2>&1 || exit 1
bash tools/ab_multi.sh cs "ab/cs0/libpldepth_hip.so pldepth_amd/libpldepth_hip.so" "dgrad 32 28 28 1344 0 240 3" "fwd 32 28 28 672 672 240 3" "fwd 32 14 14 1280 0 672 3" "dgrad 32 14 14 1280 0 672 3" "fwd 32 28 28 256 0 256 3" "fwd 32 28 28 256 0 1024 1" "dgrad 32 56 56 128 0 512 1" "fwd 32 14 14 1152 0 192 1" > /dev/null 2>&1 || exit 1
cp gpurun_out/ab_cs/ab.txt $O/ab_micro.txt
B="--no-cpu-baseline --no-loss-parity --no-extra-configs"
timeout -k 10 300 python -u bench.py $B > $O/bench_eff.json 2> $O/bench_eff.err || exit 1
PLD_LIB_PATH=ab/cs0/libpldepth_hip.so timeout -k 10 300 python -u bench.py $B > $O/bench_eff_cs0.json 2> $O/bench_eff_cs0.err || exit 1
for m in 0 1 2; do
  PLD_BN_PROLOGUE=$m timeout -k 10 300 python -u bench.py --model ff_redweb $B > $O/bench_rw_p$m.json 2> $O/bench_rw_p$m.err || exit 1
done
PLD_LIB_PATH=ab/cs0/libpldepth_hip.so PLD_BN_PROLOGUE=0 timeout -k 10 300 python -u bench.py --model ff_redweb $B > $O/bench_rw_p0_cs0.json 2> $O/bench_rw_p0_cs0.err || exit 1
timeout -k 10 300 python -u bench.py $B > $O/bench_eff2.json 2> $O/bench_eff2.err || exit 1
echo ok
