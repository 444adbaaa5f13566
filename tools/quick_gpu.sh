# quick GPU check: selected tests then a short headline bench.  bash tools/quick_gpu.sh TAG "pytest -k expr" [files]
TAG=${1:-q}
K=${2:-upconv}
shift 2
FILES=${@:-tests/test_kernels_gpu.py}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest $FILES -m gpu -x -q -k "$K" --timeout 300 --timeout-method thread > gpurun_out/${TAG}_test.log 2>&1
rc=$?
tail -15 gpurun_out/${TAG}_test.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-extra-configs > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_bench.json'));print(d['value'],d['ms_per_step'],d['loss']);print(json.dumps(d['roofline']['kernels']))"
exit $rc
