# schedule sweeps of the bench's conv shapes (graph-replayed, tools/sched_sweep.py)
set -o pipefail
O=gpurun_out/${1:-sweep}
mkdir -p $O
run() { timeout -k 10 120 python -u tools/sched_sweep.py "$@" >> $O/sweep.txt 2>&1 || { echo "FAIL $*"; tail -5 $O/sweep.txt; exit 1; }; }
run --mode fwd --h 14 --w 14 --c1 192 --k 1 --cout 1152
run --mode dgrad --h 14 --w 14 --c1 1152 --k 1 --cout 192
run --mode fwd --h 14 --w 14 --c1 1152 --k 1 --cout 192
run --mode fwd --h 28 --w 28 --c1 672 --k 1 --cout 112
run --mode fwd --h 14 --w 14 --c1 320 --k 1 --cout 1280
run --mode dgrad --h 14 --w 14 --c1 320 --k 1 --cout 1280
run --mode fwd --h 14 --w 14 --c1 1280 --k 3 --cout 672
run --mode dgrad --h 14 --w 14 --c1 1280 --k 3 --cout 672
run --mode wgrad --h 14 --w 14 --c1 1280 --k 3 --cout 672
run --mode fwd --h 28 --w 28 --c1 672 --c2 672 --k 3 --cout 240
run --mode dgrad --h 28 --w 28 --c1 672 --c2 672 --k 3 --cout 240
run --mode dgrad --h 56 --w 56 --c1 240 --c2 240 --k 3 --cout 144
echo done
