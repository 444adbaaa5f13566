#!/bin/bash
# Round-3 GPU check: the memset-node repro (packet capture on / off), the graph bisect of both
# models with the runtime's default settings, then the graph / DP / bench-N>1 tests.
set -o pipefail
O=gpurun_out/r03a
mkdir -p $O
DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 timeout -k 10 120 tools/bin/graph_memset_repro > $O/repro_pc1.txt 2>&1
echo "rc=$?" >> $O/repro_pc1.txt
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 120 tools/bin/graph_memset_repro > $O/repro_pc0.txt 2>&1
echo "rc=$?" >> $O/repro_pc0.txt
timeout -k 10 200 python -u tools/graph_bisect.py > $O/bisect_effnet.log 2>&1 || exit 1
GB_MODEL=ff_redweb timeout -k 10 200 python -u tools/graph_bisect.py > $O/bisect_redweb.log 2>&1 || exit 1
timeout -k 10 800 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_trainer_gpu.py tests/test_dp_gpu.py tests/test_bench_gpu.py > $O/tests.log 2>&1
