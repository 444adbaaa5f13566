#!/bin/bash
# GPU box: kernel tests with the generic staged epilogue (conv_x3 grid + fp32 implicit GEMM,
# routing / accumulate / sub-tile LDS regions); A/B vs the round's previous staged form (ab/stgold)
set -o pipefail
O=gpurun_out/r4s
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tk.log 2>&1 || { tail -30 $O/tk.log; exit 1; }
tail -2 $O/tk.log
for v in stgold new; do
  L=""; [ $v != new ] && L=ab/$v/libpldepth_hip.so
  for args in "--mode fwd --h 14 --w 14 --c1 192 --k 1 --cout 1152 --sched 0 1 2 3 4 5 6 7 8 9 10 11 12" "--mode dgrad --h 28 --w 28 --c1 672 --c2 672 --k 3 --cout 240 --sched 3 8 9" "--mode fwd --h 28 --w 28 --c1 672 --c2 672 --k 3 --cout 240 --sched 9" "--mode fwd --h 112 --w 112 --c1 64 --k 3 --cout 64 --math fp32 --sched 0 1 2 3 4 5 6 7 8"; do
    echo "== $v $args" >> $O/stg.txt
    PLD_LIB_PATH=$L timeout -k 10 150 python -u tools/sched_sweep.py --top 3 --n 32 $args >> $O/stg.txt 2>&1 || { echo FAIL; tail $O/stg.txt; exit 1; }
  done
done
grep -v amdgpu $O/stg.txt
for v in stgold new stgold new; do
  L=""; [ $v != new ] && L=ab/$v/libpldepth_hip.so
  PLD_LIB_PATH=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-loss-parity > $O/ab_$v.json 2> $O/ab_$v.err || { tail -20 $O/ab_$v.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/ab_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], {k: v['value'] for k, v in d.get('extra_configs', {}).items()})"
done
