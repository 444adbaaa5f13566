#!/bin/bash
# GPU box: stem (unrolled staging) + patch WGRAD XCD-order A/B (HEAD conv_x3.hip in ab/pwhead)
set -o pipefail
O=gpurun_out/r4g
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread  > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
timeout -k 10 120 python -u tools/sched_sweep.py --mode fwd --n 32 --h 448 --w 448 --c1 3 --k 3 --cout 32 --stride 2 --pad 0 --sched 0 --top 3 > $O/stem.txt 2>&1 && grep -v amdgpu.ids $O/stem.txt
for v in pwhead new; do
  L=""; [ $v != new ] && L=ab/$v/libpldepth_hip.so
  for args in "--h 56 --w 56 --c1 240 --c2 240 --cout 144" "--h 112 --w 112 --c1 144 --c2 144 --cout 32" "--h 224 --w 224 --c1 32 --cout 32"; do
    echo "== $v $args" >> $O/pw.txt
    PLD_LIB_PATH=$L timeout -k 10 150 python -u tools/sched_sweep.py --mode wgrad --n 32 --k 3 --sched 26 $args >> $O/pw.txt 2>&1 || { echo FAIL; tail $O/pw.txt; exit 1; }
  done
done
grep -v amdgpu.ids $O/pw.txt
for v in pwhead new; do
  L=$GRAFT_REPO_ROOT/ab/$v/libpldepth_hip.so; [ $v = new ] && L=""
  PLD_LIB_PATH=$L bash tools/gpu_pmc1.sh r4g/pmc_$v --mode wgrad --n 32 --k 3 --sched 26 --h 56 --w 56 --c1 240 --c2 240 --cout 144 > $O/pmc_$v.txt 2>&1 || { cat $O/pmc_$v.txt; exit 1; }
  head -2 $O/pmc_$v.txt
done
for v in epi0 new; do
  L=""; [ $v != new ] && L=ab/$v/libpldepth_hip.so
  for args in "--mode fwd --h 14 --w 14 --c1 192 --k 1 --cout 1152" "--mode dgrad --h 14 --w 14 --c1 192 --k 1 --cout 1152" "--mode fwd --h 28 --w 28 --c1 672 --k 1 --cout 112" "--mode dgrad --h 28 --w 28 --c1 112 --k 1 --cout 672" "--mode fwd --h 56 --w 56 --c1 240 --c2 240 --k 3 --cout 144" "--mode dgrad --h 28 --w 28 --c1 672 --c2 672 --k 3 --cout 240"; do
    echo "== $v $args" >> $O/s1x1.txt
    PLD_LIB_PATH=$L timeout -k 10 150 python -u tools/sched_sweep.py --top 6 --n 32 $args >> $O/s1x1.txt 2>&1 || { echo FAIL; tail $O/s1x1.txt; exit 1; }
  done
done
grep -v amdgpu.ids $O/s1x1.txt
