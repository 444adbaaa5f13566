#!/bin/bash
# One GPU session: the GPU test suite, then (unless a step faulted / timed out) the bench.
#   tools/gpu_tests_and_bench.sh TAG [pytest selection...]
# Test FAILURES (pytest exit 1) still run the bench; a crash, abort or time limit stops here.
TAG=${1:-run}
shift
SEL=${@:-tests}
mkdir -p gpurun_out
export PLD_REPORT_DIR=gpurun_out/parity_$TAG
timeout -k 10 1000 python -u -m pytest $SEL -m gpu -v -rf --timeout 300 \
    --timeout-method thread > gpurun_out/${TAG}_gputest.log 2>&1
rc=$?
tail -5 gpurun_out/${TAG}_gputest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
  echo "pytest exit $rc: stopping (no further GPU steps)"
  exit $rc
fi
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
brc=$?
tail -c 3000 gpurun_out/${TAG}_bench.json
echo "pytest exit $rc, bench exit $brc"
exit $brc
