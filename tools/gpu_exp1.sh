set -o pipefail
O=gpurun_out/${1:-exp1}
mkdir -p $O
for v in base expA expB expAB; do
  L=""; [ $v != base ] && L=ab/$v/libpldepth_hip.so
  for args in "--mode fwd --h 14 --w 14 --c1 1280 --k 3 --cout 672 --sched 5 9 3" "--mode dgrad --h 14 --w 14 --c1 1280 --k 3 --cout 672 --sched 9 3" "--mode fwd --h 14 --w 14 --c1 192 --k 1 --cout 1152 --sched 11 10"; do
    echo "== $v $args" >> $O/exp.txt
    PLD_LIB_PATH=$L timeout -k 10 120 python -u tools/sched_sweep.py $args >> $O/exp.txt 2>&1 || { echo FAIL; tail $O/exp.txt; exit 1; }
  done
done
grep -v amdgpu.ids $O/exp.txt
