set -o pipefail
O=gpurun_out/${1:-exp3}
mkdir -p $O
for v in base nostore; do
  L=""; [ $v != base ] && L=ab/$v/libpldepth_hip.so
  for args in "--mode fwd --h 14 --w 14 --c1 192 --k 1 --cout 1152" "--mode fwd --h 14 --w 14 --c1 1152 --k 1 --cout 192" "--mode fwd --h 28 --w 28 --c1 672 --k 1 --cout 112" "--mode dgrad --h 14 --w 14 --c1 1280 --k 3 --cout 672"; do
    echo "== $v $args" >> $O/exp.txt
    PLD_LIB_PATH=$L timeout -k 10 150 python -u tools/sched_sweep.py --top 4 --sched 0 1 2 3 4 5 6 7 8 9 10 11 12 $args >> $O/exp.txt 2>&1 || { echo FAIL; tail $O/exp.txt; exit 1; }
  done
done
grep -v amdgpu.ids $O/exp.txt
