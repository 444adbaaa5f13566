#!/bin/bash
# conv_micro timings of several builds of libpldepth_hip.so on the same box:
#   bash tools/ab_multi.sh TAG "lib1 lib2 ..." "mode n h w c1 c2 cout k" ...
TAG=$1; LIBS=$2; shift 2
O=gpurun_out/ab_$TAG
mkdir -p $O
for shape in "$@"; do
  set -- $shape
  for rep in 1 2; do
    for lib in $LIBS; do
      PLD_LIB_PATH=$lib timeout -k 10 60 python3 tools/conv_micro.py --mode $1 --n $2 --h $3 --w $4 --c1 $5 --c2 $6 --cout $7 --k ${8:-3} --tile -1 --iters 20 2>&1 | grep TF/s | sed "s#^#$(basename $(dirname $lib)) #" || exit 1
    done
  done
done > $O/ab.txt 2>&1
rc=$?
cat $O/ab.txt
exit $rc
