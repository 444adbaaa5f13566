"""Per-kernel HBM traffic of one training step from rocprofv3 PMC passes (tools/prof_step_pmc.sh).

    python tools/traffic.py gpurun_out/pmc_step [--marker adam_amsgrad_dev_kernel]

FETCH_SIZE is doubled (gfx950 tallies 128-B reads at 64 B: MI355X_MICROARCH.md, HBM), WRITE_SIZE
is taken as is. Uses the step window between the last two markers before bench.py's trailing
profiling step; durations come from the same passes' kernel trace.
"""
import argparse
import collections
import csv
import json
import os

CONV_MAIN = ("conv_igemm_kernel", "conv_x3_kernel", "conv_x3_patch", "thin1x1_kernel", "skinny_fwd_kernel",
             "skinny_dgrad_kernel", "skinny_wgrad_kernel")
CONV_KERNELS = CONV_MAIN + ("splitk_", "stride_scatter_kernel", "skinny_wgrad_reduce_kernel")


def load(d, counter):
    rows = list(csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))))
    out = []
    for r in rows:
        if r["Counter_Name"] != counter:
            continue
        out.append((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"]),
                    int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    out.sort()
    return out


def window(rows, marker):
    idx = [i for i, r in enumerate(rows) if marker in r[1]]
    return rows[idx[-3] + 1:idx[-2] + 1]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--marker", default="adam_amsgrad_dev_kernel")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--json", default="", help="write the conv-family summary (bench.py "
                                               "--traffic-file) here")
    a = ap.parse_args()
    f = window(load(os.path.join(a.dir, "fetch"), "FETCH_SIZE"), a.marker)
    w = window(load(os.path.join(a.dir, "write"), "WRITE_SIZE"), a.marker)
    agg = collections.defaultdict(lambda: [0, 0.0, 0.0, 0])
    for (_, name, v, d), (_, name2, v2, _) in zip(f, w):
        assert name == name2
        g = agg[name]
        g[0] += 1
        g[1] += 2 * v * 1024   # KB -> bytes, x2 read correction
        g[2] += v2 * 1024
        g[3] += d
    tot_r = sum(g[1] for g in agg.values())
    tot_w = sum(g[2] for g in agg.values())
    tot_t = sum(g[3] for g in agg.values())
    print(f"step: read {tot_r / 1e9:.2f} GB, write {tot_w / 1e9:.2f} GB, kernel time "
          f"{tot_t / 1e6:.2f} ms (PMC pass, serialized)")
    print(f"{'calls':>5} {'ms':>7} {'read GB':>8} {'write GB':>8} {'GB/s':>7}  kernel")
    for name, g in sorted(agg.items(), key=lambda kv: -kv[1][3])[:a.top]:
        bw = (g[1] + g[2]) / max(g[3], 1)
        print(f"{g[0]:5d} {g[3] / 1e6:7.3f} {g[1] / 1e9:8.3f} {g[2] / 1e9:8.3f} {bw:7.0f}  "
              f"{name[:90]}")
    if a.json:
        # the conv family as bench.py's roofline counts it: one conv call = its main kernel plus
        # the split-K / stride reductions it launches
        conv = {n: g for n, g in agg.items() if any(k in n for k in CONV_KERNELS)}
        calls = sum(g[0] for n, g in conv.items() if any(k in n for k in CONV_MAIN))
        rb = sum(g[1] for g in conv.values())
        wb = sum(g[2] for g in conv.values())
        out = {"source": a.dir, "step_read_bytes": tot_r, "step_write_bytes": tot_w,
               "conv_read_bytes_per_step": rb, "conv_write_bytes_per_step": wb,
               "conv_calls_per_step": calls,
               "conv_bytes_per_launch": round((rb + wb) / max(calls, 1)),
               "note": "FETCH_SIZE x2 (gfx950 64-B tally of 128-B reads) + WRITE_SIZE, separate "
                       "--pmc passes, eager step window between adam_amsgrad_dev_kernel markers"}
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)
        print(f"conv family: {(rb + wb) / 1e9:.2f} GB/step over {calls} calls -> {a.json}")


if __name__ == "__main__":
    main()
