#!/bin/bash
# Round-3 GPU run: memset repro (busy stream), the default bench line (loss_delta + step byte
# floor), conv tables of both models, rocprof kernel stats of the bench, PMC step traffic.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03b
mkdir -p $O
cd $R
timeout -k 10 120 tools/bin/graph_memset_repro > $O/repro_busy.txt 2>&1; echo "rc=$?" >> $O/repro_busy.txt
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 200 python -u tools/conv_table.py --math auto --top 60 > $O/conv_table_effnet.txt 2>&1 || exit 1
timeout -k 10 200 python -u tools/conv_table.py --model ff_redweb --math auto --top 60 > $O/conv_table_redweb.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extra-configs > $O/prof.log 2>&1 || exit 1
echo ok
