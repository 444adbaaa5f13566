# conv tests + wgrad sweep (GPU box)
R=$GRAFT_REPO_ROOT
M="python3 $R/tools/conv_micro.py"
O=$R/gpurun_out/exp_wgrad.txt
: > $O
timeout -k 10 300 python -u -m pytest $R/tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k conv >> $O 2>&1 || exit 1
for t in -1 0 1 3 7 8 9; do timeout -k 10 60 $M --mode wgrad --h 28 --w 28 --c1 672 --c2 672 --k 3 --cout 240 --tile $t --iters 10 >> $O 2>&1; done
for t in -1 0 1 3 7 8 9; do timeout -k 10 60 $M --mode wgrad --h 56 --w 56 --c1 240 --c2 240 --k 3 --cout 144 --tile $t --iters 10 >> $O 2>&1; done
for t in -1 0 1 7; do timeout -k 10 60 $M --mode wgrad --h 112 --w 112 --c1 144 --c2 144 --k 3 --cout 32 --tile $t --iters 5 >> $O 2>&1; done
timeout -k 10 60 $M --mode wgrad --h 14 --w 14 --c1 1280 --k 3 --cout 672 --iters 10 >> $O 2>&1
timeout -k 10 60 $M --mode wgrad --h 224 --w 224 --c1 32 --k 3 --cout 32 --iters 5 >> $O 2>&1
echo done >> $O
