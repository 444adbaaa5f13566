"""Per-family HBM traffic of one training step from the rocprofv3 PMC passes of
tools/prof_step_pmc.sh (FETCH_SIZE and WRITE_SIZE in separate runs, eager steps): the measured
side of bench.py's step-level byte floor (roofline.step_bytes_algorithmic).

    python tools/pmc_step_family.py gpurun_out/pmc_step --workload "<bench workload string>" \
        --json profiles/r03_pmc_step_family.json

FETCH_SIZE x2 (gfx950 tallies 128-B reads at 64 B: MI355X_MICROARCH.md, HBM) + WRITE_SIZE, step
window between the last adam_amsgrad_dev_kernel markers (tools/traffic.py)."""
import argparse
import collections
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from traffic import load, window  # noqa: E402

# kernel name -> op family (bench._family names the same families by kernels.py wrapper)
FAMILIES = [
    ("sampler_listmle", ("listmle_kernel", "mean_kernel", "zero_kernel", "compact_", "draw_kernel",
                         "candidate", "select_", "copy_first_kernel")),
    ("optimizer_refresh", ("adam_amsgrad", "filter_native", "filter_dgrad", "step_increment",
                           "set_scalar")),
    ("batchnorm", ("bn_apply", "bn_bwd_apply", "bn_infer", "chan_reduce", "stats_finalize",
                   "bnbwd_finalize", "sum_finalize")),
    ("depthwise", ("dw_fwd_tile", "dwconv_")),
    ("squeeze_excite", ("img_chan_sum", "se_fc_")),
    ("resample_residual", ("upsample2x", "maxpool", "residual", "dropconnect")),
    ("conv", ("conv_x3", "conv_igemm", "thin1x1", "wide1x1", "pgemm", "skinny", "scalar1x1",
              "splitk_", "stride_scatter", "upconv", "filter_split")),
]


def family_of(kernel):
    for fam, keys in FAMILIES:
        if any(k in kernel for k in keys):
            return fam
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--workload", required=True)
    ap.add_argument("--marker", default="adam_amsgrad_dev_kernel")
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    f = window(load(os.path.join(a.dir, "fetch"), "FETCH_SIZE"), a.marker)
    w = window(load(os.path.join(a.dir, "write"), "WRITE_SIZE"), a.marker)
    fam = collections.defaultdict(lambda: [0.0, 0.0, 0, 0])
    for (_, name, v, d), (_, name2, v2, _) in zip(f, w):
        assert name == name2
        g = fam[family_of(name)]
        g[0] += 2 * v * 1024
        g[1] += v2 * 1024
        g[2] += 1
        g[3] += d
    tot = sum(g[0] + g[1] for g in fam.values())
    for k, g in sorted(fam.items(), key=lambda kv: -(kv[1][0] + kv[1][1])):
        print(f"{k:20s} {g[2]:4d} launches  read {g[0] / 1e9:7.3f} GB  write {g[1] / 1e9:7.3f} GB"
              f"  {g[3] / 1e6:7.3f} ms  {(g[0] + g[1]) / max(g[3], 1):6.0f} GB/s")
    print(f"total {tot / 1e9:.3f} GB")
    if a.json:
        out = {"workload": a.workload, "source": a.dir, "total_bytes": tot,
               "by_family": {k: round(g[0] + g[1]) for k, g in fam.items()},
               "by_family_detail": {k: {"read": round(g[0]), "write": round(g[1]),
                                        "launches": g[2], "ms_serialized": g[3] / 1e6}
                                    for k, g in fam.items()}}
        with open(a.json, "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
