# conv kernel A/B on the GPU box: the conv parity tests, the isolated decoder conv shapes and the
# per-conv table of one training step.   bash tools/conv_ab.sh TAG
TAG=${1:-x}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "conv" --timeout 300 --timeout-method thread > gpurun_out/${TAG}_convtest.log 2>&1 || { tail -30 gpurun_out/${TAG}_convtest.log; exit 1; }
tail -2 gpurun_out/${TAG}_convtest.log
timeout -k 10 200 python -u tools/conv_shapes_bench.py > gpurun_out/${TAG}_shapes.txt 2>&1 || exit 1
cat gpurun_out/${TAG}_shapes.txt
timeout -k 10 300 python -u tools/conv_table.py --math auto --top 25 > gpurun_out/${TAG}_table.txt 2>&1 || exit 1
tail -28 gpurun_out/${TAG}_table.txt
