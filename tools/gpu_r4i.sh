#!/bin/bash
# GPU box: kernel tests; patch-WGRAD tap-group A/B (ab/pwtg1 = one consumer wave per SIMD); BN
# in-kernel finalize A/B (ab/bnhead = finalize kernels); schedule table re-tune; full GPU suite
set -o pipefail
O=gpurun_out/r4i
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tk.log 2>&1 || { tail -30 $O/tk.log; exit 1; }
tail -2 $O/tk.log
bash tools/gpu_r4j.sh || exit 1
bash tools/gpu_r4k.sh || exit 1
for v in pwtg1 new; do
  L=""; [ $v != new ] && L=ab/$v/libpldepth_hip.so
  for args in "--h 56 --w 56 --c1 240 --c2 240 --cout 144" "--h 112 --w 112 --c1 144 --c2 144 --cout 32" "--h 224 --w 224 --c1 32 --cout 32" "--h 28 --w 28 --c1 672 --c2 672 --cout 240"; do
    echo "== $v $args" >> $O/pw.txt
    PLD_LIB_PATH=$L timeout -k 10 150 python -u tools/sched_sweep.py --mode wgrad --n 32 --k 3 --sched 26 $args >> $O/pw.txt 2>&1 || { echo FAIL; tail $O/pw.txt; exit 1; }
  done
done
grep -v amdgpu.ids $O/pw.txt
for v in bnhead new; do
  L=""; [ $v != new ] && L=ab/$v/libpldepth_hip.so
  PLD_LIB_PATH=$L timeout -k 10 300 python -u tools/bn_table.py --top 45 > $O/bn_$v.txt 2>&1 || { tail -20 $O/bn_$v.txt; exit 1; }
  tail -5 $O/bn_$v.txt
done
timeout -k 10 600 python -u bench.py --tune pldepth_amd/schedules/gfx950.json --no-cpu-baseline --no-loss-parity > $O/tune.json 2> $O/tune.err || { tail -20 $O/tune.err; exit 1; }
tail -c 300 $O/tune.json; echo
sha1sum pldepth_amd/schedules/gfx950.json
export PLD_REPORT_DIR=$O/parity
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
rc=$?
tail -5 $O/gputest.log
exit $rc
