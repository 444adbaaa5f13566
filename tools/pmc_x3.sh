# PMC passes for conv_x3 shapes (GPU box): bash tools/pmc_x3.sh TAG
R=$GRAFT_REPO_ROOT
TAG=${1:-x}
cd /tmp && export TMPDIR=/tmp
run() {
  name=$1; shift
  O=$R/gpurun_out/pmc_${TAG}_$name
  mkdir -p $O
  C1="python3 $R/tools/conv_micro.py $* --iters 5"
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY --kernel-trace -d $O/p1 -o run --output-format csv -- $C1 > $O/p1.log 2>&1 || return 1
  timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --kernel-trace -d $O/p2 -o run --output-format csv -- $C1 > $O/p2.log 2>&1 || return 1
  grep "TF/s" $O/p1.log | tail -1
  python3 $R/tools/pmc_summary.py $O conv_x3
}
run dec0_dgrad --mode dgrad --n 32 --h 14 --w 14 --c1 1280 --c2 0 --k 3 --cout 672 --tile 9 || exit 1
run dec1_fwd --mode fwd --n 32 --h 28 --w 28 --c1 672 --c2 672 --k 3 --cout 240 --tile 9 || exit 1
run dec0_wgrad --mode wgrad --n 32 --h 14 --w 14 --c1 1280 --c2 0 --k 3 --cout 672 --tile 1 || exit 1
echo done
