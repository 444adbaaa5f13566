"""Decoder 3x3 convs (ff_effnet, batch 32, 448x448) on the row-band halo kernel vs the schedule
the persisted table picks (round 6): per shape and mode, ms / TF/s of the table's schedule and of
every x3halo / x3halosplit schedule, and each halo result's max relative difference from the
table schedule's output.

    python tools/halo_ab.py [--iters 20] [--only dec0,dec1,dec2] [--modes fwd,dgrad]
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHAPES = {"dec0": (14, 14, 1280, 0, 672), "dec1": (28, 28, 672, 672, 240),
          "dec2": (56, 56, 240, 240, 144)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--n", type=int, default=32)
    ap.add_argument("--only", default="dec0,dec1,dec2")
    ap.add_argument("--modes", default="fwd,dgrad")
    ap.add_argument("--scheds", default="", help="comma list of schedule names (default: all halo)")
    a = ap.parse_args()
    from pldepth_amd import kernels as K
    from pldepth_amd._lib import lib
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    K.use_schedule_table()
    m = K.MATH["bf16x3"]
    names = [lib().pld_conv_schedule_desc(m, i).decode()
             for i in range(lib().pld_conv_num_schedules(m))]
    halo = [s for s in names if s.startswith("x3halo")]
    if a.scheds:
        halo = a.scheds.split(",")
    g = torch.Generator(device=dev).manual_seed(0)
    for name in a.only.split(","):
        h, w, c1, c2, cout = SHAPES[name]
        x1 = torch.randn(a.n, h, w, c1, device=dev, generator=g)
        x2 = torch.randn(a.n, h, w, c2, device=dev, generator=g) if c2 else None
        C = c1 + c2
        wt = torch.randn(3, 3, C, cout, device=dev, generator=g) / (9 * C) ** 0.5
        wn, wd = K.filter_to_native(wt), K.filter_to_dgrad(wt)
        K.filter_split(wn, torch.empty_like(wn))
        K.filter_split(wd, torch.empty_like(wd))
        y = torch.empty(a.n, h, w, cout, device=dev)
        dy = torch.randn(a.n, h, w, cout, device=dev, generator=g)
        dx1, dx2 = torch.empty_like(x1), (torch.empty_like(x2) if c2 else None)
        for mode in a.modes.split(","):
            fl = 2.0 * a.n * h * w * cout * 9 * C
            args = K.conv_args(x1, x2, 3, 3, 1, 1, 1, h, w, cout, math="bf16x3")

            def run():
                if mode == "fwd":
                    K.conv2d_fwd(args, wn, None, y)
                    return y
                K.conv2d_dgrad(args, dy, wd, dx1, dx2)
                return torch.cat([dx1.flatten()] + ([dx2.flatten()] if c2 else []))

            def timed(tile):
                args.tile = tile
                ref = run().clone()
                torch.cuda.synchronize()
                best = float("inf")
                for _ in range(3):
                    e0, e1 = (torch.cuda.Event(enable_timing=True),
                              torch.cuda.Event(enable_timing=True))
                    e0.record()
                    for _ in range(a.iters):
                        run()
                    e1.record()
                    e1.synchronize()
                    best = min(best, e0.elapsed_time(e1) / a.iters)
                return best, ref

            key = K._shape_key(mode, args)
            t0 = K._TILE_CACHE.get(key, -1)
            base_ms, base = timed(t0)
            print(f"{name} {mode}: table {K.schedule_desc(m, t0)} {base_ms:.3f} ms "
                  f"{fl / base_ms / 1e9:.0f} TF/s", flush=True)
            for s in halo:
                idx = K._schedule_index(m, s)
                ms, out = timed(idx)
                d = float((out - base).abs().max() / base.abs().max())
                print(f"    {s:22s} {ms:.3f} ms {fl / ms / 1e9:5.0f} TF/s  "
                      f"x{base_ms / ms:.2f}  maxrel {d:.2e}", flush=True)


if __name__ == "__main__":
    main()
