# conv tests + tile sweep of the bf16x3 conv on the decoder's heaviest shapes (GPU box)
R=$GRAFT_REPO_ROOT
M="python3 $R/tools/conv_micro.py"
O=$R/gpurun_out/exp_tiles.txt
: > $O
timeout -k 10 300 python -u -m pytest $R/tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k conv >> $O 2>&1 || exit 1
for t in 3 9 8 4 13 19; do timeout -k 10 60 $M --mode fwd --h 14 --w 14 --c1 1280 --k 3 --cout 672 --tile $t --iters 10 >> $O 2>&1; done
for t in 3 9 8 4 13 19; do timeout -k 10 60 $M --mode fwd --h 28 --w 28 --c1 672 --c2 672 --k 3 --cout 240 --tile $t --iters 10 >> $O 2>&1; done
for t in 3 9 8 13 19; do timeout -k 10 60 $M --mode dgrad --h 28 --w 28 --c1 672 --c2 672 --k 3 --cout 240 --tile $t --iters 10 >> $O 2>&1; done
timeout -k 10 60 $M --mode fwd --h 28 --w 28 --c1 12096 --k 1 --cout 256 --tile 9 --iters 10 >> $O 2>&1
timeout -k 10 60 $M --mode fwd --h 112 --w 112 --c1 144 --c2 144 --k 3 --cout 32 --iters 10 >> $O 2>&1
timeout -k 10 60 $M --mode fwd --h 56 --w 56 --c1 240 --c2 240 --k 3 --cout 144 --iters 10 >> $O 2>&1
echo done >> $O
