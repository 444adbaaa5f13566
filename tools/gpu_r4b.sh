set -o pipefail
O=gpurun_out/r4b
mkdir -p $O
timeout -k 10 300 python -u tools/conv_table.py --math auto --top 100 --schedules pldepth_amd/schedules/gfx950.json > $O/conv_table.txt 2>&1
rc=$?; echo "table rc=$rc"; tail -3 $O/conv_table.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u tools/exp_dec_precision.py --schedules pldepth_amd/schedules/gfx950.json --out $O/exp.json > $O/exp.log 2>&1
rc=$?; tail -12 $O/exp.log; exit $rc
