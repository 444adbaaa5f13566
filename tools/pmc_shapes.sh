# MFMA / LDS / wait counters for a few bf16x3 conv shapes (GPU box): bash tools/pmc_shapes.sh
R=$GRAFT_REPO_ROOT
run() {  # name, conv_micro args
  n=$1; shift
  mkdir -p $R/gpurun_out/pmcs/$n
  cd /tmp && export TMPDIR=/tmp
  C1="python3 $R/tools/conv_micro.py $* --iters 5"
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY --kernel-trace -d $R/gpurun_out/pmcs/$n/p1 -o run --output-format csv -- $C1 > $R/gpurun_out/pmcs/$n/p1.log 2>&1 || return 1
  timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --kernel-trace -d $R/gpurun_out/pmcs/$n/p2 -o run --output-format csv -- $C1 > $R/gpurun_out/pmcs/$n/p2.log 2>&1 || return 1
  python3 $R/tools/conv_micro.py $* --iters 20 > $R/gpurun_out/pmcs/$n/time.txt 2>&1
}
run fwd_big --mode fwd --n 32 --h 28 --w 28 --c1 672 --c2 672 --k 3 --cout 240 --math bf16x3 || exit 1
run dgrad_big --mode dgrad --n 32 --h 14 --w 14 --c1 1280 --c2 0 --k 3 --cout 672 --math bf16x3 || exit 1
run fwd_n32 --mode fwd --n 32 --h 112 --w 112 --c1 144 --c2 144 --k 3 --cout 32 --math bf16x3 || exit 1
run wgrad_n32 --mode wgrad --n 32 --h 112 --w 112 --c1 144 --c2 144 --k 3 --cout 32 --math bf16x3 || exit 1
echo done
