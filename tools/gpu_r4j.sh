#!/bin/bash
# GPU box: store cache-policy experiment on the BN apply kernel (ab/st1 = sc1 write-through
# 16-B stores, ab/st2 = nt 16-B stores, new = plain): back-to-back launches incl. boundaries
set -o pipefail
O=gpurun_out/r4j
mkdir -p $O
for v in new st1 st2; do
  L=""; [ $v != new ] && L=ab/$v/libpldepth_hip.so
  for sh in "--rows 401408 --c 144" "--rows 100352 --c 240" "--rows 25088 --c 672" "--rows 6272 --c 1152"; do
    echo "== $v $sh" >> $O/st.txt
    PLD_LIB_PATH=$L timeout -k 10 120 python -u tools/bn_micro.py $sh --iters 30 >> $O/st.txt 2>&1 || { tail $O/st.txt; exit 1; }
  done
done
grep -v amdgpu.ids $O/st.txt
