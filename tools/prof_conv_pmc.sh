# conv microbenchmarks + PMC passes for the bf16x3 conv kernel (run on the GPU box)
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
M="python3 $R/tools/conv_micro.py"
: > $R/gpurun_out/pmc/micro.txt
for t in -1 3 6 9 16 19; do timeout -k 10 60 $M --mode fwd --h 14 --w 14 --c1 1280 --cout 672 --tile $t --iters 10 >> $R/gpurun_out/pmc/micro.txt 2>&1; done
for t in -1 3 9 13 19; do timeout -k 10 60 $M --mode fwd --h 28 --w 28 --c1 672 --c2 672 --cout 240 --tile $t --iters 10 >> $R/gpurun_out/pmc/micro.txt 2>&1; done
timeout -k 10 60 $M --mode dgrad --h 28 --w 28 --c1 672 --c2 672 --cout 240 --iters 10 >> $R/gpurun_out/pmc/micro.txt 2>&1
timeout -k 10 60 $M --mode wgrad --h 28 --w 28 --c1 672 --c2 672 --cout 240 --iters 10 >> $R/gpurun_out/pmc/micro.txt 2>&1
timeout -k 10 60 $M --mode fwd --h 112 --w 112 --c1 144 --c2 0 --cout 144 --iters 10 >> $R/gpurun_out/pmc/micro.txt 2>&1
C1="$M --mode fwd --h 14 --w 14 --c1 1280 --cout 672 --tile 6 --iters 10"
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY --kernel-trace -d $R/gpurun_out/pmc/p1 -o run --output-format csv -- $C1 > $R/gpurun_out/pmc/p1.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --kernel-trace -d $R/gpurun_out/pmc/p2 -o run --output-format csv -- $C1 > $R/gpurun_out/pmc/p2.log 2>&1
echo done
