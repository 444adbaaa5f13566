"""HBM traffic of the bench line's dominant conv kernel, beside its algorithmic bytes.

    python tools/dominant_traffic.py gpurun_out/pmc_step BENCH_JSON OUT_PREFIX

PMC side: FETCH_SIZE (x2, gfx950 tallies 128-B reads at 64 B — MI355X_MICROARCH.md) and
WRITE_SIZE from the separate passes of tools/prof_step_pmc.sh, one eager step window between
adam_amsgrad_dev_kernel markers, summed over every launch whose name is the dominant kernel
(any template instance). Algorithmic side: the bench line's roofline.dominant (bytes_per_step /
launches_per_step: each operand read once, the output written once). Writes OUT_PREFIX.txt
(human readable) and OUT_PREFIX.json (read by bench.py to fill roofline.traffic when its own
workload and dominant kernel match).
"""
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import traffic as T  # noqa: E402


def short(name):
    m = re.search(r"([A-Za-z_][A-Za-z_0-9]*)\s*[<(]", name.replace("void ", "", 1))
    return m.group(1) if m else name


def main():
    pmc, bench_file, out = sys.argv[1:4]
    line = [ln for ln in open(bench_file) if ln.startswith("{")][-1]
    b = json.loads(line)
    dom = b["roofline"]["dominant"]
    kname = dom["kernel"]
    f = T.window(T.load(os.path.join(pmc, "fetch"), "FETCH_SIZE"), "adam_amsgrad_dev_kernel")
    w = T.window(T.load(os.path.join(pmc, "write"), "WRITE_SIZE"), "adam_amsgrad_dev_kernel")
    rows = []
    for (_, n1, v1, d), (_, n2, v2, _) in zip(f, w):
        assert n1 == n2
        if short(n1.split("::")[-1]) == kname or short(n1) == kname:
            rows.append((n1, 2 * v1 * 1024, v2 * 1024, d))
    if not rows:
        raise SystemExit(f"no launches of {kname} in the PMC window")
    n = len(rows)
    rd = sum(r[1] for r in rows)
    wr = sum(r[2] for r in rows)
    algo = dom["bytes_per_step"]
    res = {
        "kernel": kname, "workload": b["config"]["workload"],
        "launches_pmc": n, "launches_bench": dom["launches_per_step"],
        "hbm_read_bytes_per_step": rd, "hbm_write_bytes_per_step": wr,
        "hbm_bytes_per_launch": round((rd + wr) / n),
        "algorithmic_bytes_per_step": algo,
        "algorithmic_bytes_per_launch": round(algo / dom["launches_per_step"]),
        "hbm_over_algorithmic": round((rd + wr) / algo, 3),
        "source": pmc, "bench_line": bench_file,
        "note": "FETCH_SIZE x2 + WRITE_SIZE, separate --pmc passes, one eager step",
    }
    mdir = os.path.join(pmc, "mfma")
    if os.path.isdir(mdir):
        # MFMA busy share: SQ_VALU_MFMA_BUSY_CYCLES (cycles, summed over the 1024 SIMDs) over the
        # launches' own cycles (GRBM_GUI_ACTIVE, summed over the 8 XCDs: / 8), same launches
        mb = T.window(T.load(mdir, "SQ_VALU_MFMA_BUSY_CYCLES"), "adam_amsgrad_dev_kernel")
        gr = T.window(T.load(mdir, "GRBM_GUI_ACTIVE"), "adam_amsgrad_dev_kernel")
        busy = cyc = 0.0
        for (_, n1, v1, _), (_, n2, v2, _) in zip(mb, gr):
            if short(n1.split("::")[-1]) == kname or short(n1) == kname:
                busy += v1
                cyc += v2 / 8
        if cyc > 0:
            res["mfma_busy"] = round(busy / (1024 * cyc), 4)
    with open(out + ".json", "w") as fh:
        json.dump(res, fh, indent=1)
    with open(out + ".txt", "w") as fh:
        fh.write(f"dominant kernel: {kname}  (bench workload: {res['workload']})\n")
        fh.write(f"launches per step: PMC {n}, bench {dom['launches_per_step']}\n")
        fh.write(f"HBM per step (PMC): read {rd / 1e9:.3f} GB, write {wr / 1e9:.3f} GB\n")
        fh.write(f"HBM per launch: {res['hbm_bytes_per_launch'] / 1e6:.2f} MB; algorithmic per "
                 f"launch: {res['algorithmic_bytes_per_launch'] / 1e6:.2f} MB; ratio "
                 f"{res['hbm_over_algorithmic']}\n")
        if "mfma_busy" in res:
            fh.write(f"MFMA busy (SQ_VALU_MFMA_BUSY_CYCLES / SIMD cycles): {res['mfma_busy']}\n")
        fh.write(f"{'read MB':>9} {'write MB':>9} {'us':>8}  launch\n")
        for name, r_, w_, d in rows:
            fh.write(f"{r_ / 1e6:9.2f} {w_ / 1e6:9.2f} {d / 1e3:8.1f}  {name[:110]}\n")
    print(open(out + ".txt").read())


if __name__ == "__main__":
    main()
