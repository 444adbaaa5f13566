#!/bin/bash
# GPU box: BN-backward reduction variants (residual specialisation, occupancy, grid size):
# BN kernel tests on the in-tree build (v1), micro timings and an alternating step A/B
set -o pipefail
O=gpurun_out/r4u
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "bn or reduc" --timeout 120 --timeout-method thread > $O/tk.log 2>&1 || { tail -30 $O/tk.log; exit 1; }
tail -2 $O/tk.log
for v in base v1 v2 v3; do
  L=""; [ $v != v1 ] && L=ab/$v/libpldepth_hip.so
  for sh in "--rows 401408 --c 144 --act swish" "--rows 1605632 --c 96 --act swish" "--rows 100352 --c 240 --act swish" "--rows 401408 --c 64 --act relu"; do
    PLD_LIB_PATH=$L timeout -k 10 120 python -u tools/bn_micro.py $sh --iters 20 > $O/micro.txt 2>&1 || { tail -20 $O/micro.txt; exit 1; }
    echo "$v $(tail -1 $O/micro.txt)" | tee -a $O/micro_all.txt
  done
done
for v in base v1 v2 v3 base v1 v2 v3; do
  L=""; [ $v != v1 ] && L=ab/$v/libpldepth_hip.so
  PLD_LIB_PATH=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-loss-parity --no-extra-configs > $O/ab_$v.json 2> $O/ab_$v.err || { tail -20 $O/ab_$v.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/ab_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'])" | tee -a $O/step_ab.txt
done
