#!/bin/bash
# GPU box: SE squeeze grid A/B (ab/se2048: 2048 workgroups, ab/seru8: 8 rows of loads in flight)
set -o pipefail
O=gpurun_out/r4o
mkdir -p $O
for v in new se2048 seru8 new; do
  L=""; [ $v != new ] && L=ab/$v/libpldepth_hip.so
  echo "== $v" >> $O/se.txt
  PLD_LIB_PATH=$L timeout -k 10 200 python -u tools/se_micro.py --iters 20 >> $O/se.txt 2>&1 || { tail $O/se.txt; exit 1; }
done
grep -v amdgpu $O/se.txt
