# A/B of conv_micro shapes between ab/base/libpldepth_hip.so and the in-tree build (GPU box):
#   bash tools/ab_micro.sh TAG "mode n h w c1 c2 cout k acc" ...
TAG=$1; shift
O=gpurun_out/ab_$TAG
mkdir -p $O
for shape in "$@"; do
  set -- $shape
  for lib in ab/base/libpldepth_hip.so pldepth_amd/libpldepth_hip.so; do
    for rep in 1 2; do
      PLD_LIB_PATH=$lib timeout -k 10 60 python3 tools/conv_micro.py --mode $1 --n $2 --h $3 --w $4 --c1 $5 --c2 $6 --cout $7 --k ${8:-3} --acc ${9:-0} --tile -1 --iters 20 2>&1 | grep TF/s | sed "s#^#$(basename $(dirname $lib)) acc=${9:-0} #" || exit 1
    done
  done
done > $O/ab.txt 2>&1
rc=$?
cat $O/ab.txt
exit $rc
