#!/bin/bash
# GPU box: kernel tests with the LDS-staged nt-store grid epilogue, then the step A/B against the
# previous library (ab/epiold)
set -o pipefail
O=gpurun_out/r4q
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tk.log 2>&1 || { tail -30 $O/tk.log; exit 1; }
tail -2 $O/tk.log
for v in epiold new epiold new; do
  L=""; [ $v != new ] && L=ab/$v/libpldepth_hip.so
  PLD_LIB_PATH=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-loss-parity > $O/ab_$v.json 2> $O/ab_$v.err || { tail -20 $O/ab_$v.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/ab_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], {k: v['value'] for k, v in d.get('extra_configs', {}).items()})"
done
