# rocprofv3 kernel trace + --stats of the 1-GPU bench (graph-replayed steps), and the per-step
# window of it (tools/kstats.py: the last STEPS steps between Adam launches, the trailing eager
# profiling step dropped). GPU box: bash tools/prof_bench.sh TAG [STEPS]
R=$GRAFT_REPO_ROOT
TAG=${1:-x}
STEPS=${2:-8}
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python3 $R/bench.py --steps $STEPS --warmup 3 --no-cpu-baseline --no-extra-configs > $O/bench.log 2>&1 || exit 1
DB=$(ls $O/trace/*/run_results.db 2>/dev/null | head -1)
[ -z "$DB" ] && DB=$(ls $O/trace/run_results.db 2>/dev/null | head -1)
python3 $R/tools/kstats.py $DB --marker adam_amsgrad_dev_kernel --steps $STEPS --skip 1 --csv $O/kernel_stats.csv --top 60 > $O/kstats.txt
cp $(ls $O/trace/*/run_kernel_stats.csv $O/trace/run_kernel_stats.csv 2>/dev/null | head -1) $O/rocprof_stats_native.csv 2>/dev/null
tail -c 400 $O/bench.log
head -70 $O/kstats.txt
