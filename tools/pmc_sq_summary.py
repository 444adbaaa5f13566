"""Per-kernel SQ counter summary of tools/pmc_step_sq.sh: last eager step's dispatches of each
kernel name, counters summed over its dispatches, with derived ratios:
  mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (duration x 2.4 GHz x 1024 SIMDs)
  lds_active = SQ_LDS_IDX_ACTIVE / (duration x 2.4 GHz x 256 CUs)
  wait_any / wave_cycles, wait_inst_lds / wave_cycles."""
import collections
import csv
import glob
import sys

O = sys.argv[1]
cnt = collections.defaultdict(lambda: collections.defaultdict(float))
dur = {}
name = {}
for p in ("p1", "p2"):
    cc = glob.glob(f"{O}/{p}/**/run_counter_collection.csv", recursive=True)
    kt = glob.glob(f"{O}/{p}/**/run_kernel_trace.csv", recursive=True)
    if not cc:
        continue
    # the step's dispatches are the last ones of each kernel name (warm-up step first)
    rows = list(csv.DictReader(open(cc[0])))
    ids = sorted({int(r["Dispatch_Id"]) for r in rows})
    half = ids[len(ids) // 2:] if len(ids) > 1 else ids
    keep = set(half)
    for r in rows:
        d = int(r["Dispatch_Id"])
        if d in keep:
            cnt[(p, d)][r["Counter_Name"]] += float(r["Counter_Value"])
            name[(p, d)] = r["Kernel_Name"].split("(")[0]
    if kt:
        for r in csv.DictReader(open(kt[0])):
            d = int(r["Dispatch_Id"])
            if d in keep:
                dur[(p, d)] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for key, c in cnt.items():
    n = name[key]
    for k, v in c.items():
        agg[n][k] += v
    agg[n]["dur_" + key[0]] += dur.get(key, 0.0)
    agg[n]["n_" + key[0]] += 1
for n, a in sorted(agg.items(), key=lambda kv: -kv[1].get("dur_p2", 0.0)):
    d2 = a.get("dur_p2", 0.0) or 1e-30
    d1 = a.get("dur_p1", 0.0) or 1e-30
    out = {"launches": int(a.get("n_p2", 0)), "ms": round(d2 * 1e3, 3)}
    if "SQ_VALU_MFMA_BUSY_CYCLES" in a:
        out["mfma_busy"] = round(a["SQ_VALU_MFMA_BUSY_CYCLES"] / (d2 * 2.4e9 * 1024), 3)
    if "SQ_LDS_IDX_ACTIVE" in a:
        out["lds_active"] = round(a["SQ_LDS_IDX_ACTIVE"] / (d2 * 2.4e9 * 256), 3)
        out["lds_conflict_frac"] = round(a["SQ_LDS_BANK_CONFLICT"] / max(a["SQ_LDS_IDX_ACTIVE"], 1), 3)
    if "SQ_WAVE_CYCLES" in a:
        wc = max(a["SQ_WAVE_CYCLES"], 1)
        out["wait_any"] = round(a["SQ_WAIT_ANY"] / wc, 3)
        out["wait_inst_lds"] = round(a["SQ_WAIT_INST_LDS"] / wc, 3)
        out["insts_per_wave"] = {k: round(a[k] / max(a["SQ_WAVES"], 1), 1)
                                 for k in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_MFMA")}
    if "SQ_ACTIVE_INST_ANY" in a and "SQ_WAIT_INST_ANY" in a:
        out["valu_active"] = round(a["SQ_ACTIVE_INST_VALU"] / max(a["SQ_ACTIVE_INST_ANY"] + a["SQ_WAIT_INST_ANY"], 1), 3)
    out["raw"] = {k: a[k] for k in sorted(a) if k.startswith(("SQ_", "GRBM"))}
    print(n, out)
