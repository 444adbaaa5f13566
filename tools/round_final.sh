# Round-end evidence (GPU box): full GPU test suite, default bench line (with cpu_baseline),
# rocprofv3 kernel trace + per-step kstats, PMC traffic of one eager step + the dominant kernel's
# HBM vs algorithmic bytes, ff_redweb kernel trace. bash tools/round_final.sh TAG [--no-tests]
TAG=${1:-final}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
rc=0
# progress marker for the GPU pool's silence watchdog (a parity test's fp64 oracle runs
# several minutes without printing); every step below keeps its own time limit
(while sleep 45; do date >> $O/heartbeat.txt; done) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
if [ "$2" != "--no-tests" ]; then
  export PLD_REPORT_DIR=$O/parity
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
  rc=$?
  tail -3 $O/gputest.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python3 $R/bench.py > $O/bench.json 2> $O/bench.err || exit 1
tail -c 600 $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extra-configs > $O/trace.log 2>&1 || exit 1
DB=$(ls $O/trace/*/run_results.db 2>/dev/null | head -1)
[ -z "$DB" ] && DB=$(ls $O/trace/run_results.db 2>/dev/null | head -1)
python3 $R/tools/kstats.py $DB --marker adam_amsgrad_dev_kernel --steps 10 --skip 1 --csv $O/kernel_stats.csv --top 70 > $O/kstats.txt || exit 1
cp $(ls $O/trace/*/run_kernel_stats.csv $O/trace/run_kernel_stats.csv 2>/dev/null | head -1) $O/rocprof_stats_native.csv 2>/dev/null
head -3 $O/kstats.txt
bash $R/tools/prof_step_pmc.sh > $O/pmc.log 2>&1 || exit 1
python3 $R/tools/traffic.py $R/gpurun_out/pmc_step > $O/pmc_traffic.txt 2>&1
python3 $R/tools/dominant_traffic.py $R/gpurun_out/pmc_step $O/bench.json $O/pmc_dominant > $O/dom.log 2>&1
cat $O/dom.log | tail -5
WL="ff_effnet train step 448x448, per-GPU batch 32, ranking_size 5, rankings_per_image 100, sampler info, Adam-AMSGrad"
python3 $R/tools/pmc_step_family.py $R/gpurun_out/pmc_step --workload "$WL" --json $O/pmc_step_family.json > $O/pmc_step_family.txt 2>&1
python3 $R/tools/dominant_graph.py $O/kernel_stats.csv 10 $O/dominant_graph.json --bench $O/bench.json --source "profiles/${TAG}_kernel_stats.csv (rocprofv3 --kernel-trace of bench.py, 10 graph-replay steps, tools/kstats.py)" > /dev/null 2>&1
rm -rf $O/trace
bash $R/tools/prof_redweb.sh ${TAG}_rw > /dev/null 2>&1 || exit 1
head -3 $R/gpurun_out/prof_${TAG}_rw/kstats.txt
echo done
exit $rc
