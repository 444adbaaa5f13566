#!/bin/bash
# GPU box: the BN-backward SE squeeze grid (1024 base / 768 / 1536 workgroups): SE tests on the
# in-tree build, the squeeze's per-launch time in a rocprofv3 kernel trace of the bench step per
# variant, then an alternating step A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4v
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "se or squeeze" --timeout 120 --timeout-method thread > $O/tk.log 2>&1 || { tail -30 $O/tk.log; exit 1; }
tail -2 $O/tk.log
cd /tmp && export TMPDIR=/tmp
for v in base b768 b1536; do
  L=""; [ $v != base ] && L=$R/ab/$v/libpldepth_hip.so
  PLD_LIB_PATH=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tr_$v -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extra-configs --no-loss-parity > $O/tr_$v.log 2>&1 || { tail -20 $O/tr_$v.log; exit 1; }
  DB=$(find $O/tr_$v -name "*.db" | head -1)
  python3 $R/tools/kstats.py $DB --marker adam_amsgrad_dev_kernel --steps 10 --skip 1 --csv $O/stats_$v.csv --top 70 > $O/kstats_$v.txt || exit 1
  { echo "== $v"; head -2 $O/kstats_$v.txt; grep -E "img_chan_sum|se_fc_bwd|bnbwd_finalize|bn_bwd_apply" $O/kstats_$v.txt || true; } | tee -a $O/stats.txt
  rm -rf $O/tr_$v
done
cd $R
for v in b768 base b768 base; do
  L=""; [ $v != base ] && L=ab/$v/libpldepth_hip.so
  PLD_LIB_PATH=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-loss-parity --no-extra-configs > $O/ab_$v.json 2> $O/ab_$v.err || { tail -20 $O/ab_$v.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/ab_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'])" | tee -a $O/step_ab.txt
done
