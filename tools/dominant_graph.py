"""The dominant conv kernel's per-step time in graph replay, from a tools/kstats.py CSV of a
rocprofv3 kernel trace of bench.py (the file bench.py --graph-profile reads).

    python tools/dominant_graph.py KERNEL_STATS.csv STEPS OUT.json [--kernel NAME | --bench BENCH.json]

Sums every instantiation of the kernel (all tile / mode template arguments) over the window's
STEPS steps; the workload string is bench.py's default cfg2 one. The kernel: --kernel, else the
bench line's roofline.kernel (--bench), else conv_x3_kernel."""
import argparse
import csv
import json

WORKLOAD = ("ff_effnet train step 448x448, per-GPU batch 32, ranking_size 5, "
            "rankings_per_image 100, sampler info, Adam-AMSGrad")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("steps", type=int)
    ap.add_argument("out")
    ap.add_argument("--kernel", default="")
    ap.add_argument("--bench", default="", help="bench.py JSON line: its dominant kernel")
    ap.add_argument("--source", default="")
    a = ap.parse_args()
    if not a.kernel and a.bench:
        with open(a.bench) as f:
            a.kernel = json.loads(f.read().strip().splitlines()[-1])["roofline"]["kernel"]
    a.kernel = a.kernel or "conv_x3_kernel"
    calls = ns = 0
    with open(a.csv) as f:
        for row in csv.DictReader(f):
            name = row["Name"]
            base = name.split("<")[0].split("(")[0].split("::")[-1]
            if base == a.kernel:
                calls += int(row["Calls"])
                ns += int(row["TotalDurationNs"])
    assert calls % a.steps == 0, (calls, a.steps)
    out = {"kernel": a.kernel, "workload": WORKLOAD,
           "ms_per_step": round(ns / a.steps / 1e6, 4),
           "launches_per_step": calls // a.steps,
           "source": a.source or f"{a.csv} (rocprofv3 --kernel-trace of bench.py, {a.steps} "
                                 "graph-replay steps, tools/kstats.py)"}
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
