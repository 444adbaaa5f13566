# uniform-wave x3 tiles vs the autotuned schedule on the big decoder convs (GPU box)
#   bash tools/exp_uni.sh TAG
TAG=${1:-u}
O=gpurun_out/uni_$TAG
mkdir -p $O
run() {  # mode n h w c1 c2 cout
  for t in -1 10 11 12 13 24 25 26 27; do
    timeout -k 10 60 python3 tools/conv_micro.py --mode $1 --n $2 --h $3 --w $4 --c1 $5 --c2 $6 --k 3 --cout $7 --tile $t --iters 10 2>&1 | grep TF/s || return 1
  done
}
{
run dgrad 32 28 28 672 672 240 &&
run fwd 32 56 56 240 240 144 &&
run dgrad 32 56 56 240 240 144 &&
run fwd 32 28 28 672 672 240 &&
run fwd 32 14 14 1280 0 672 &&
run dgrad 32 112 112 144 144 32 &&
run dgrad 32 14 14 1280 0 672
} > $O/micro.txt 2>&1
rc=$?
cat $O/micro.txt
exit $rc
