R=$GRAFT_REPO_ROOT
M="python3 $R/tools/conv_micro.py"
O=$R/gpurun_out/exp1.txt
: > $O
timeout -k 10 60 $M --mode fwd --h 14 --w 14 --c1 1280 --k 3 --cout 672 --iters 10 >> $O 2>&1
timeout -k 10 60 $M --mode fwd --h 14 --w 14 --c1 11520 --k 1 --cout 672 --iters 10 >> $O 2>&1
timeout -k 10 60 $M --mode fwd --h 28 --w 28 --c1 672 --c2 672 --k 3 --cout 240 --iters 10 >> $O 2>&1
timeout -k 10 60 $M --mode fwd --h 28 --w 28 --c1 12096 --k 1 --cout 240 --iters 10 >> $O 2>&1
timeout -k 10 60 $M --mode fwd --h 28 --w 28 --c1 12096 --k 1 --cout 256 --iters 10 >> $O 2>&1
timeout -k 10 60 $M --mode fwd --h 56 --w 56 --c1 4096 --k 1 --cout 256 --iters 10 >> $O 2>&1
timeout -k 10 60 $M --mode fwd --h 112 --w 112 --c1 2592 --k 1 --cout 32 --iters 10 >> $O 2>&1
timeout -k 10 60 $M --mode fwd --h 112 --w 112 --c1 144 --c2 144 --k 3 --cout 32 --iters 10 >> $O 2>&1
echo done >> $O
