#!/bin/bash
# GPU box: 8 consumer waves (two per SIMD) on the occupancy-1 bf16x3 tiles (ab/w8) vs 4 (new)
set -o pipefail
O=gpurun_out/r4k
mkdir -p $O
for v in new w8; do
  L=""; [ $v != new ] && L=ab/$v/libpldepth_hip.so
  for args in "--mode fwd --h 14 --w 14 --c1 1280 --k 3 --cout 672" "--mode dgrad --h 14 --w 14 --c1 1280 --k 3 --cout 672" "--mode fwd --h 28 --w 28 --c1 672 --c2 672 --k 3 --cout 240" "--mode dgrad --h 28 --w 28 --c1 672 --c2 672 --k 3 --cout 240" "--mode wgrad --h 14 --w 14 --c1 1280 --k 3 --cout 672"; do
    echo "== $v $args" >> $O/w8.txt
    S="3 8 9 21 22 37 38"; case "$args" in *wgrad*) S="3 8 9 37 38";; esac
    PLD_LIB_PATH=$L timeout -k 10 150 python -u tools/sched_sweep.py --top 8 --n 32 --sched $S $args >> $O/w8.txt 2>&1 || { echo FAIL; tail $O/w8.txt; exit 1; }
  done
done
grep -v amdgpu.ids $O/w8.txt
