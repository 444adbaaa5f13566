# PMC passes for one bf16x3 conv launch shape (GPU box): bash tools/prof_conv_pmc.sh <conv_micro args>
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
C1="python3 $R/tools/conv_micro.py $*"
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY --kernel-trace -d $R/gpurun_out/pmc/p1 -o run --output-format csv -- $C1 > $R/gpurun_out/pmc/p1.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --kernel-trace -d $R/gpurun_out/pmc/p2 -o run --output-format csv -- $C1 > $R/gpurun_out/pmc/p2.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $R/gpurun_out/pmc/p3 -o run --output-format csv -- $C1 > $R/gpurun_out/pmc/p3.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d $R/gpurun_out/pmc/p4 -o run --output-format csv -- $C1 > $R/gpurun_out/pmc/p4.log 2>&1
echo done
