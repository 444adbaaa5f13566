set -o pipefail
O=gpurun_out/${1:-exp2}
mkdir -p $O
for v in base pipe0; do
  L=""; [ $v != base ] && L=ab/$v/libpldepth_hip.so
  for args in "--mode fwd --h 14 --w 14 --c1 1280 --k 3 --cout 672" "--mode dgrad --h 14 --w 14 --c1 1280 --k 3 --cout 672" "--mode wgrad --h 14 --w 14 --c1 1280 --k 3 --cout 672" "--mode fwd --h 28 --w 28 --c1 672 --c2 672 --k 3 --cout 240" "--mode dgrad --h 28 --w 28 --c1 672 --c2 672 --k 3 --cout 240" "--mode dgrad --h 56 --w 56 --c1 240 --c2 240 --k 3 --cout 144" "--mode fwd --h 14 --w 14 --c1 192 --k 1 --cout 1152"; do
    echo "== $v $args" >> $O/exp.txt
    PLD_LIB_PATH=$L timeout -k 10 150 python -u tools/sched_sweep.py --top 14 --sched 0 1 2 3 4 5 6 7 8 9 10 11 12 $args >> $O/exp.txt 2>&1 || { echo FAIL; tail $O/exp.txt; exit 1; }
  done
done
echo done
