set -o pipefail
O=gpurun_out/r4a
mkdir -p $O
timeout -k 10 900 python -u bench.py --tune $O/gfx950.json --no-cpu-baseline > $O/bench_tune.json 2> $O/bench_tune.err
rc=$?; echo "bench rc=$rc"; tail -c 600 $O/bench_tune.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/diag_dec_wgrad.py --schedules $O/gfx950.json > $O/diag.txt 2>&1
rc=$?; echo "diag rc=$rc"; cat $O/diag.txt | tail -8; [ $rc -ne 0 ] && exit $rc
timeout -k 10 700 python -u -m pytest tests/test_bench_gpu.py -x -v --timeout 600 --timeout-method thread > $O/t.log 2>&1
rc=$?; tail -5 $O/t.log; exit $rc
