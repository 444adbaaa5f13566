#!/bin/bash
# GPU box: grid-epilogue store policy A/B (timing only): new = per-element C-layout stores;
# epi1/2/3 = LDS-staged 16-B row stores, plain / write-through (sc1) / streaming (nt)
set -o pipefail
O=gpurun_out/r4p
mkdir -p $O
for v in new epi1 epi2 epi3; do
  L=""; [ $v != new ] && L=ab/$v/libpldepth_hip.so
  for args in "--mode fwd --h 14 --w 14 --c1 192 --k 1 --cout 1152" "--mode dgrad --h 14 --w 14 --c1 192 --k 1 --cout 1152" "--mode fwd --h 28 --w 28 --c1 672 --k 1 --cout 112" "--mode dgrad --h 28 --w 28 --c1 112 --k 1 --cout 672" "--mode fwd --h 56 --w 56 --c1 144 --k 1 --cout 24" "--mode fwd --h 28 --w 28 --c1 672 --c2 672 --k 3 --cout 240"; do
    echo "== $v $args" >> $O/epi.txt
    PLD_LIB_PATH=$L timeout -k 10 150 python -u tools/sched_sweep.py --top 3 --n 32 --sched 0 1 2 3 4 5 6 7 8 9 10 11 12 $args >> $O/epi.txt 2>&1 || { echo FAIL; tail $O/epi.txt; exit 1; }
  done
done
grep -v amdgpu $O/epi.txt
