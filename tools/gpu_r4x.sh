#!/bin/bash
# GPU box: BN-backward reduction grid for the ReLU / swish instances (3 workgroups per CU):
# 2048 (base, in-tree) vs 768 (one round). BN tests on both, micro timings, kernel trace, step A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4x
mkdir -p $O
for v in base r768; do
  L=""; [ $v != base ] && L=ab/$v/libpldepth_hip.so
  PLD_LIB_PATH=$L timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "bn or reduc" --timeout 120 --timeout-method thread > $O/tk_$v.log 2>&1 || { tail -30 $O/tk_$v.log; exit 1; }
  echo "$v $(tail -1 $O/tk_$v.log)"
  for sh in "--rows 401408 --c 144 --act swish" "--rows 1605632 --c 96 --act swish" "--rows 100352 --c 240 --act swish" "--rows 401408 --c 64 --act relu"; do
    PLD_LIB_PATH=$L timeout -k 10 120 python -u tools/bn_micro.py $sh --iters 20 > $O/micro.txt 2>&1 || { tail -20 $O/micro.txt; exit 1; }
    echo "$v $(tail -1 $O/micro.txt)" | tee -a $O/micro_all.txt
  done
done
cd /tmp && export TMPDIR=/tmp
for v in base r768; do
  L=""; [ $v != base ] && L=$R/ab/$v/libpldepth_hip.so
  PLD_LIB_PATH=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tr_$v -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extra-configs --no-loss-parity > $O/tr_$v.log 2>&1 || { tail -20 $O/tr_$v.log; exit 1; }
  DB=$(find $O/tr_$v -name "*.db" | head -1)
  python3 $R/tools/kstats.py $DB --marker adam_amsgrad_dev_kernel --steps 10 --skip 1 --csv $O/stats_$v.csv --top 70 > $O/kstats_$v.txt || exit 1
  { echo "== $v"; head -2 $O/kstats_$v.txt; grep -E "chan_reduce|bnbwd_finalize|bn_bwd_apply" $O/kstats_$v.txt || true; } | tee -a $O/stats.txt
  rm -rf $O/tr_$v
done
cd $R
for v in r768 base r768 base r768 base; do
  L=""; [ $v != base ] && L=ab/$v/libpldepth_hip.so
  PLD_LIB_PATH=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-loss-parity --no-extra-configs > $O/ab_$v.json 2> $O/ab_$v.err || { tail -20 $O/ab_$v.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/ab_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'])" | tee -a $O/step_ab.txt
done
