#!/bin/bash
# rocprof kernel stats of the tiled-dgrad build vs ab/base (HEAD dwtile + dwse)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r03z
mkdir -p $O
B="--no-cpu-baseline --no-loss-parity --no-extra-configs"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_new -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 $B > $R/$O/prof_new.log 2>&1 || exit 1
PLD_LIB_PATH=$R/ab/base/libpldepth_hip.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_base -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 $B > $R/$O/prof_base.log 2>&1 || exit 1
echo ok
