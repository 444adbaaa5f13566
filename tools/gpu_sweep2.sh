set -o pipefail
O=gpurun_out/${1:-sweep2}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "tile_stream or conv_every_schedule" > $O/t.log 2>&1 || { tail -20 $O/t.log; exit 1; }
tail -2 $O/t.log
run() { timeout -k 10 120 python -u tools/sched_sweep.py --top 60 "$@" >> $O/sweep.txt 2>&1 || { echo "FAIL $*"; tail -5 $O/sweep.txt; exit 1; }; }
run --mode fwd --h 14 --w 14 --c1 1280 --k 3 --cout 672
run --mode wgrad --h 14 --w 14 --c1 1280 --k 3 --cout 672
run --mode fwd --h 28 --w 28 --c1 672 --c2 672 --k 3 --cout 240
echo done
