#!/bin/bash
# (1) kernel tests: pgemm with the channel quad fixed per thread, every conv schedule incl. the
# new 64x64 bf16x3 tile, the conv prologue; (2) ff_effnet bench: current build vs HEAD pgemm
# (ab/pg_old) vs HEAD conv_x3 (ab/x3_head, no 64x64 tile); (3) ff_redweb conv input prologue
# A/B per PLD_BN_PROLOGUE mode (0 off, 1 conv2+conv3, 2 conv3 only, 3 conv2 only) + conv tables.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r03n
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "pgemm or every_schedule or prologue or conv_fwd_dgrad" > $O/tests.log 2>&1 || exit 1
B="--no-cpu-baseline --no-loss-parity --no-extra-configs"
timeout -k 10 300 python -u bench.py $B > $O/bench_eff.json 2> $O/bench_eff.err || exit 1
PLD_LIB_PATH=ab/pg_old/libpldepth_hip.so timeout -k 10 300 python -u bench.py $B > $O/bench_eff_pgold.json 2> $O/bench_eff_pgold.err || exit 1
PLD_LIB_PATH=ab/x3_head/libpldepth_hip.so timeout -k 10 300 python -u bench.py $B > $O/bench_eff_x3head.json 2> $O/bench_eff_x3head.err || exit 1
for m in 0 1 2 3; do
  PLD_BN_PROLOGUE=$m timeout -k 10 300 python -u bench.py --model ff_redweb $B > $O/bench_rw_p$m.json 2> $O/bench_rw_p$m.err || exit 1
done
PLD_LIB_PATH=ab/x3_head/libpldepth_hip.so PLD_BN_PROLOGUE=0 timeout -k 10 300 python -u bench.py --model ff_redweb $B > $O/bench_rw_p0_x3head.json 2> $O/bench_rw_p0_x3head.err || exit 1
PLD_BN_PROLOGUE=1 timeout -k 10 200 python -u tools/conv_table.py --model ff_redweb --math auto --top 200 > $O/conv_table_rw_p1.txt 2>&1 || exit 1
PLD_BN_PROLOGUE=0 timeout -k 10 200 python -u tools/conv_table.py --model ff_redweb --math auto --top 200 > $O/conv_table_rw_p0.txt 2>&1 || exit 1
timeout -k 10 200 python -u tools/conv_table.py --model ff_effnet --math auto --top 200 > $O/conv_table_eff.txt 2>&1 || exit 1
echo ok
