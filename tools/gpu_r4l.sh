#!/bin/bash
# GPU box: kernel tests; step A/B of the nt BN-apply stores (ab/plainst = plain stores); schedule
# table re-tune (written under gpurun_out, copied into the tree afterwards); full GPU suite
set -o pipefail
O=gpurun_out/r4l
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tk.log 2>&1 || { tail -30 $O/tk.log; exit 1; }
tail -2 $O/tk.log
for sh in "--rows 401408 --c 144 --act swish" "--rows 401408 --c 256 --act relu"; do
  PMC_KRE="chan_reduce_kernel<2" PMC_TOOL=tools/bn_micro.py bash tools/gpu_pmc1.sh r4l/pmc_bn_$(echo $sh | tr -dc 0-9a-z | head -c 20) $sh --iters 5 > $O/pmc_bn.txt 2>&1 || { cat $O/pmc_bn.txt; exit 1; }
  echo "== $sh" >> $O/pmc_bn_all.txt; cat $O/pmc_bn.txt >> $O/pmc_bn_all.txt
done
head -4 $O/pmc_bn_all.txt
for v in plainst new plainst new; do
  L=""; [ $v != new ] && L=ab/$v/libpldepth_hip.so
  PLD_LIB_PATH=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-loss-parity --no-extra-configs > $O/ab_$v.json 2> $O/ab_$v.err || { tail -20 $O/ab_$v.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/ab_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'])"
done
for v in plainst new; do
  L=""; [ $v != new ] && L=ab/$v/libpldepth_hip.so
  PLD_LIB_PATH=$L timeout -k 10 300 python -u tools/bn_table.py --top 45 > $O/bn_$v.txt 2>&1 || { tail -20 $O/bn_$v.txt; exit 1; }
  tail -5 $O/bn_$v.txt
done
timeout -k 10 600 python -u bench.py --tune $O/gfx950.json --no-cpu-baseline --no-loss-parity > $O/tune.json 2> $O/tune.err || { tail -20 $O/tune.err; exit 1; }
cp $O/gfx950.json pldepth_amd/schedules/gfx950.json && sha1sum pldepth_amd/schedules/gfx950.json
export PLD_REPORT_DIR=$O/parity
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
rc=$?
tail -5 $O/gputest.log
exit $rc
