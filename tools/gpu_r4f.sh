#!/bin/bash
# GPU box: stem kernel tests + conv dispatch tests, then the epilogue (no-store) experiment
set -o pipefail
O=gpurun_out/r4f
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "stem3x3 or bn_stats or prologue" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -3 $O/t.log
timeout -k 10 120 python -u tools/sched_sweep.py --mode fwd --n 32 --h 448 --w 448 --c1 3 --k 3 --cout 32 --stride 2 --pad 0 --sched 0 --top 3 > $O/stem.txt 2>&1 && cat $O/stem.txt
bash tools/gpu_exp3.sh r4f
