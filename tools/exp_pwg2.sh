# patch WGRAD A/B on the decoder shapes (GPU box): bash tools/exp_pwg2.sh TAG
TAG=${1:-w}
O=gpurun_out/pwg_$TAG
mkdir -p $O
{
for t in -1 20; do
timeout -k 10 60 python3 tools/conv_micro.py --mode wgrad --n 32 --h 56 --w 56 --c1 240 --c2 240 --k 3 --cout 144 --tile $t --iters 10 2>&1 | grep TF/s &&
timeout -k 10 60 python3 tools/conv_micro.py --mode wgrad --n 32 --h 112 --w 112 --c1 144 --c2 144 --k 3 --cout 32 --tile $t --iters 10 2>&1 | grep TF/s &&
timeout -k 10 60 python3 tools/conv_micro.py --mode wgrad --n 32 --h 224 --w 224 --c1 32 --c2 0 --k 3 --cout 32 --tile $t --iters 10 2>&1 | grep TF/s &&
timeout -k 10 60 python3 tools/conv_micro.py --mode wgrad --n 32 --h 28 --w 28 --c1 672 --c2 672 --k 3 --cout 240 --tile $t --iters 10 2>&1 | grep TF/s || exit 1
done
} > $O/micro.txt 2>&1
rc=$?
cat $O/micro.txt
exit $rc
