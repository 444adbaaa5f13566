# GPU: selected tests, then the rocprof kernel-trace step profile (tools/prof_bench.sh).
#   bash tools/gpu_check_prof.sh TAG "pytest -k expr" files...
TAG=${1:-c}
K=${2:-dwconv}
shift 2
FILES=${@:-tests/test_kernels_gpu.py}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest $FILES -m gpu -x -q -k "$K" --timeout 300 --timeout-method thread > gpurun_out/${TAG}_test.log 2>&1
rc=$?
tail -4 gpurun_out/${TAG}_test.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/prof_bench.sh $TAG 8 > gpurun_out/${TAG}_prof.log 2>&1 || { tail gpurun_out/${TAG}_prof.log; exit 1; }
head -3 gpurun_out/prof_$TAG/kstats.txt
grep -E "dw_fwd|dwconv|chan_reduce|bn_|stats_final|img_chan|pgemm|thin" gpurun_out/prof_$TAG/kstats.txt | head -30
