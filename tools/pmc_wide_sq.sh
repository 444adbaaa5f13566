# SQ counters of the wide 1x1 kernel on one tools/wide_ab.py shape (GPU box):
#   bash tools/pmc_wide_sq.sh SHAPE_INDEX [BIG]
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
export WIDE_AB_ONLY=$1 WIDE_AB_REPS=5
[ -n "$2" ] && export WIDE_AB_BIG=1
O=$R/gpurun_out/pmcsq_wide_$1$2
mkdir -p $O
C1="python3 $R/tools/wide_ab.py"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY --kernel-trace -d $O/p1 -o run --output-format csv -- $C1 > $O/p1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --kernel-trace -d $O/p2 -o run --output-format csv -- $C1 > $O/p2.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_EXP --kernel-trace -d $O/p3 -o run --output-format csv -- $C1 > $O/p3.log 2>&1 || echo "pass 3 failed"
python3 $R/tools/pmc_summary.py $O wide1x1
