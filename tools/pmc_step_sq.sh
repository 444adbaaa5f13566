# SQ counters (MFMA busy, LDS activity, waits) of the conv_x3 kernels of one eager training step,
# the bench schedule table. GPU box: bash tools/pmc_step_sq.sh [regex]
RX=${1:-conv_x3}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_sq
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-extra-configs --no-graph"
timeout -k 10 200 $B > $O/warm.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --kernel-include-regex "$RX" --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY --kernel-trace -d $O/p1 -o run --output-format csv -- $B > $O/p1.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --kernel-include-regex "$RX" --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --kernel-trace -d $O/p2 -o run --output-format csv -- $B > $O/p2.log 2>&1 || exit 1
python3 $R/tools/pmc_sq_summary.py $O
