# rocprofv3 kernel trace of the ff_redweb (cfg3) bench, per-step window (GPU box):
#   bash tools/prof_redweb.sh TAG [STEPS]
R=$GRAFT_REPO_ROOT
TAG=${1:-rw}
STEPS=${2:-4}
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python3 $R/bench.py --model ff_redweb --steps $STEPS --warmup 2 --no-cpu-baseline --no-extra-configs > $O/bench.log 2>&1 || exit 1
DB=$(ls $O/trace/*/run_results.db 2>/dev/null | head -1)
[ -z "$DB" ] && DB=$(ls $O/trace/run_results.db 2>/dev/null | head -1)
python3 $R/tools/kstats.py $DB --marker adam_amsgrad_dev_kernel --steps $STEPS --skip 1 --csv $O/kernel_stats.csv --top 60 > $O/kstats.txt
rm -rf $O/trace
tail -c 300 $O/bench.log
head -45 $O/kstats.txt
