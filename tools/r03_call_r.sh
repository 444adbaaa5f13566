#!/bin/bash
# Widened-input stems (ff_effnet: 4 channels, exact fp32 vector path; ff_redweb: 8 channels,
# bf16x3 under auto; PLD_STEM_PAD=0 = the scalar 3-channel path): kernel + whole-model tests,
# both benches per mode; SE backward squeeze with one sigmoid per element vs HEAD (ab/se_old).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r03r
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "stem or bn or pgemm or se_" > $O/tests.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/se_micro.py > $O/se_new.txt 2>&1 || exit 1
PLD_LIB_PATH=ab/se_old/libpldepth_hip.so timeout -k 10 120 python -u tools/se_micro.py > $O/se_old.txt 2>&1 || exit 1
PLD_REPORT_DIR=$O/parity timeout -k 10 900 python -u -m pytest -v --timeout 600 --timeout-method thread tests/test_configs_gpu.py tests/test_model_gpu.py tests/test_redweb_gpu.py > $O/model_tests.log 2>&1
rc=$?; echo "rc=$rc" >> $O/model_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
B="--no-cpu-baseline --no-loss-parity --no-extra-configs"
for m in 4 0; do
  PLD_STEM_PAD=$m timeout -k 10 300 python -u bench.py $B > $O/bench_eff_s$m.json 2> $O/bench_eff_s$m.err || exit 1
done
for m in 8 0; do
  PLD_STEM_PAD=$m timeout -k 10 300 python -u bench.py --model ff_redweb $B > $O/bench_rw_s$m.json 2> $O/bench_rw_s$m.err || exit 1
done
echo ok
