# HBM traffic of the wide 1x1 kernel on one tools/wide_ab.py shape (GPU box):
#   bash tools/pmc_wide.sh SHAPE_INDEX [BIG]
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
export WIDE_AB_ONLY=$1 WIDE_AB_REPS=5
[ -n "$2" ] && export WIDE_AB_BIG=1
O=$R/gpurun_out/pmc_wide_$1$2
mkdir -p $O
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/f -o run --output-format csv -- python3 $R/tools/wide_ab.py > $O/f.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/w -o run --output-format csv -- python3 $R/tools/wide_ab.py > $O/w.log 2>&1 || exit 1
python3 - $O <<'PY'
import csv, glob, sys, collections
o = sys.argv[1]
for c in ("f", "w"):
    f = glob.glob(f"{o}/{c}/**/run_counter_collection.csv", recursive=True)[0]
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"][:60]].append((float(r["Counter_Value"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    for k, v in agg.items():
        print(c, k, len(v), "avg KB %.0f" % (sum(x for x, _ in v) / len(v)), "avg us %.1f" % (sum(d for _, d in v) / len(v) / 1e3))
PY
