# HBM traffic per kernel of the training step: FETCH_SIZE and WRITE_SIZE in separate passes
# (rocprofv3 --pmc, kernel trace) + an MFMA-busy pass, eager steps, the bench's schedule table. Usage (GPU box): bash tools/prof_step_pmc.sh [model]
MODEL=${1:-ff_effnet}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc_step
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --model $MODEL --steps 2 --warmup 1 --no-cpu-baseline --no-extra-configs --no-graph"
timeout -k 10 200 $B > $R/gpurun_out/pmc_step/warm.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $R/gpurun_out/pmc_step/fetch -o run --output-format csv -- $B > $R/gpurun_out/pmc_step/fetch.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $R/gpurun_out/pmc_step/write -o run --output-format csv -- $B > $R/gpurun_out/pmc_step/write.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $R/gpurun_out/pmc_step/mfma -o run --output-format csv -- $B > $R/gpurun_out/pmc_step/mfma.log 2>&1
echo done
