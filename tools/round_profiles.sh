# Round-end evidence on the GPU box: default bench line (with cpu_baseline), a rocprofv3
# kernel-trace of the bench, PMC HBM-traffic passes of one eager step, and the ff_redweb bench.
# Usage (GPU box): bash tools/round_profiles.sh   -> gpurun_out/round/
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/round
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python3 $R/bench.py > $O/bench_effnet.json 2> $O/bench_effnet.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/trace.log 2>&1 || exit 1
timeout -k 10 300 python3 $R/bench.py --model ff_redweb --no-cpu-baseline > $O/bench_redweb.json 2> $O/bench_redweb.err || exit 1
bash $R/tools/prof_step_pmc.sh > $O/pmc.log 2>&1 || exit 1
echo done
