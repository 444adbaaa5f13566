set -o pipefail
O=gpurun_out/r4e
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 300 --timeout-method thread -k "conv_every_schedule or tile_stream or bn_stats_gemm_epilogue or prologue_every" > $O/t.log 2>&1
rc=$?; tail -5 $O/t.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u bench.py --tune $O/gfx950.json --no-cpu-baseline > $O/bench_tune.json 2> $O/bench_tune.err
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && { tail -20 $O/bench_tune.err; exit $rc; }
python -c "
import json; d=json.loads(open('$O/bench_tune.json').read().strip().splitlines()[-1]); r=d['roofline']
print(d['value'], d['ms_per_step'], r['kernel'], r['frac'], {k: d['extra_configs'][k]['value'] for k in d.get('extra_configs', {})})"
timeout -k 10 300 python -u tools/conv_table.py --math auto --top 100 --schedules $O/gfx950.json > $O/conv_table.txt 2>&1
echo table rc=$?
