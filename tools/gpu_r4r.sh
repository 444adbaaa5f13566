#!/bin/bash
# GPU box: kernel tests with the patch-conv LDS epilogue; patch fwd/dgrad A/B (ab/patchold);
# step A/B
set -o pipefail
O=gpurun_out/r4r
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tk.log 2>&1 || { tail -30 $O/tk.log; exit 1; }
tail -2 $O/tk.log
for v in patchold new; do
  L=""; [ $v != new ] && L=ab/$v/libpldepth_hip.so
  for args in "--mode fwd --h 112 --w 112 --c1 32 --k 3 --cout 32" "--mode dgrad --h 224 --w 224 --c1 32 --k 3 --cout 32" "--mode dgrad --h 112 --w 112 --c1 144 --c2 144 --k 3 --cout 32"; do
    echo "== $v $args" >> $O/patch.txt
    PLD_LIB_PATH=$L timeout -k 10 150 python -u tools/sched_sweep.py --top 3 --n 32 --sched 26 27 28 $args >> $O/patch.txt 2>&1 || { echo FAIL; tail $O/patch.txt; exit 1; }
  done
done
grep -v amdgpu $O/patch.txt
for v in patchold new patchold new; do
  L=""; [ $v != new ] && L=ab/$v/libpldepth_hip.so
  PLD_LIB_PATH=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-loss-parity --no-extra-configs > $O/ab_$v.json 2> $O/ab_$v.err || { tail -20 $O/ab_$v.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/ab_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'])"
done
