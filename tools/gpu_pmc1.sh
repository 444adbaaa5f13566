# SQ / TCC counters of one conv schedule (tools/sched_sweep.py --sched), separate passes.
# PMC_KRE: kernel-name regex (default the bf16x3 conv kernels); PMC_TOOL: the program under the
# profiler (default tools/sched_sweep.py), given the remaining arguments
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-pmc1}
shift
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
KRE=${PMC_KRE:-conv_x3|x3_stream}
B="python3 $GRAFT_REPO_ROOT/${PMC_TOOL:-tools/sched_sweep.py} $*"
i=0
for C in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE" \
         "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-include-regex "$KRE" --pmc $C --kernel-trace -d $O/p$i -o run --output-format csv -- $B > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
python3 - "$O" "$KRE" <<'PY'
import csv, glob, re, sys, collections
O = sys.argv[1]
kre = re.compile(sys.argv[2])
tot = collections.defaultdict(float); n = collections.Counter(); dur = collections.defaultdict(float)
for p in sorted(glob.glob(O + "/p*/")):
    cc = glob.glob(p + "**/run_counter_collection.csv", recursive=True)
    kt = glob.glob(p + "**/run_kernel_trace.csv", recursive=True)
    if not cc: continue
    rows = list(csv.DictReader(open(cc[0])))
    for r in rows:
        tot[r["Counter_Name"]] += float(r["Counter_Value"])
    for r in csv.DictReader(open(kt[0])):
        if kre.search(r["Kernel_Name"]):
            dur[p] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9; n[p] += 1
d = sum(dur.values()) / max(len(dur), 1); k = max(n.values())
print("dispatches per pass", k, "avg us", d / k * 1e6)
wc = tot["SQ_WAVE_CYCLES"]
print({"mfma_busy": tot["SQ_VALU_MFMA_BUSY_CYCLES"] / (d * 2.4e9 * 1024), "wait_any": tot["SQ_WAIT_ANY"] / wc,
       "wait_inst_any": tot["SQ_WAIT_INST_ANY"] / wc, "wait_inst_lds": tot["SQ_WAIT_INST_LDS"] / wc,
       "lds_active": tot["SQ_LDS_IDX_ACTIVE"] / (d * 2.4e9 * 256),
       "fetch_MB_per_launch": 2 * tot["FETCH_SIZE"] * 1024 / k / 1e6, "write_MB_per_launch": tot["WRITE_SIZE"] * 1024 / k / 1e6,
       "l2_hit": tot["TCC_HIT_sum"] / max(tot["TCC_HIT_sum"] + tot["TCC_MISS_sum"], 1),
       "busy_clk_MHz": tot["GRBM_GUI_ACTIVE"] / 8 / d / 1e6})
print({kk: v / k for kk, v in sorted(tot.items())})
PY
