"""Per-kernel statistics from a rocprofv3 kernel-trace SQLite database (rocpd schema).

    python tools/kstats.py gpurun_out/prof/run_results.db|<csv dir> [--csv out.csv] [--top N]
        [--marker adam_amsgrad_dev_kernel --steps 8 --skip 1]

With --marker, only dispatches inside the last `steps` marker-to-marker windows (dropping the
last `skip` markers, e.g. bench.py's trailing eager profiling step) are counted, so one-off work
(conv schedule tuning, graph capture) stays out of per-step figures; totals are then per step.
"""
import argparse
import csv
import sqlite3
import sys


def load(db):
    """(name, start, end) per dispatch from a rocpd SQLite database, a rocprofv3 csv output
    directory (its *kernel_trace.csv) or that csv file."""
    import glob
    import os
    if os.path.isdir(db):
        db = sorted(glob.glob(os.path.join(db, "*kernel_trace.csv")))[0]
    if db.endswith(".csv"):
        with open(db) as f:
            rows = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
                    for r in csv.DictReader(f)]
        return sorted(rows, key=lambda r: r[1])
    c = sqlite3.connect(db)
    return c.execute("select name, start, end from kernels order by start").fetchall()


def window(rows, marker, steps, skip):
    idx = [i for i, r in enumerate(rows) if marker in r[0]]
    if len(idx) < steps + 1 + skip:
        raise SystemExit(f"only {len(idx)} '{marker}' dispatches")
    end = idx[len(idx) - 1 - skip]
    begin = idx[len(idx) - 1 - skip - steps]
    return rows[begin + 1:end + 1]


def stats(rows):
    agg = {}
    for name, s, e in rows:
        a = agg.setdefault(name, [0, 0, 1 << 62, 0])
        d = e - s
        a[0] += 1
        a[1] += d
        a[2] = min(a[2], d)
        a[3] = max(a[3], d)
    total = sum(a[1] for a in agg.values())
    out = []
    for name, (n, t, mn, mx) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        out.append((name, n, t, t / n, 100.0 * t / total, mn, mx))
    return out, total


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv", default="")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--marker", default="")
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--skip", type=int, default=1)
    a = ap.parse_args()
    rows = load(a.db)
    per = 1
    if a.marker:
        rows = window(rows, a.marker, a.steps, a.skip)
        per = a.steps
        wall = (rows[-1][2] - rows[0][1]) / per
        print(f"window: {a.steps} steps, {len(rows) // per} dispatches/step, "
              f"wall {wall / 1e6:.3f} ms/step")
    out, total = stats(rows)
    if a.marker:
        # GPU busy time = union of all kernel intervals (the step runs on 2-3 streams); the rest
        # of the wall is idle: kernel boundaries, launch gaps, dependency waits
        busy, cur_s, cur_e = 0, None, None
        for _, s0, e0 in sorted(rows, key=lambda r: r[1]):
            if cur_e is None or s0 > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                cur_s, cur_e = s0, e0
            else:
                cur_e = max(cur_e, e0)
        busy += cur_e - cur_s
        wall_ns = rows[-1][2] - rows[0][1]
        print(f"gpu busy {busy / per / 1e6:.3f} ms/step (union of kernel intervals), idle "
              f"{(wall_ns - busy) / per / 1e6:.3f} ms/step = {100.0 * (wall_ns - busy) / wall_ns:.1f} %"
              f" of the wall")
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs",
                        "MaxNs"])
            for r in out:
                w.writerow([r[0], r[1], r[2], f"{r[3]:.1f}", f"{r[4]:.2f}", r[5], r[6]])
    print(f"kernel time {total / 1e6 / per:.3f} ms per step")
    for r in out[:a.top]:
        print(f"{r[4]:6.2f}% {r[2] / 1e6 / per:8.3f} ms/step {r[1] / per:7.1f} x "
              f"{r[3] / 1e3:9.1f} us  {r[0][:100]}")


if __name__ == "__main__":
    sys.exit(main())
