"""Merge the row-band halo schedules into the persisted conv schedule table (round 6): for every
table entry the halo kernel can take (fwd / dgrad, 3x3 stride 1 'same', maps up to 56 wide),
time the entry's schedule and every x3halo* schedule on that shape in isolation (best of 3 runs
of --iters launches, a drained device, random data) and keep the fastest when it beats the
entry by more than --margin. Other entries are left as they are (a whole re-tune moves many
unrelated choices by timing noise: profiles/r05_retune_ab.txt).

    python tools/halo_tune.py [--table pldepth_amd/schedules/gfx950.json] [--out PATH]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--table", default="")
    ap.add_argument("--out", default="")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--margin", type=float, default=0.02)
    a = ap.parse_args()
    from pldepth_amd import kernels as K
    from pldepth_amd._lib import lib
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    table = a.table or K.DEFAULT_SCHEDULES
    K.use_schedule_table(table)
    m = K.MATH["bf16x3"]
    halo = [i for i in range(lib().pld_conv_num_schedules(m))
            if lib().pld_conv_schedule_class(m, i) == 6]
    g = torch.Generator(device=dev).manual_seed(0)
    report = []
    for key in sorted(K._TILE_CACHE, key=str):
        mode, n, h, w, c1, c2, kh, kw, sh, sw, pt, pl, oh, ow, cout, pro, math = key
        if math != m or pro or mode == "wgrad":
            continue
        x1 = torch.randn(n, h, w, c1, device=dev, generator=g)
        x2 = torch.randn(n, h, w, c2, device=dev, generator=g) if c2 else None
        args = K.conv_args(x1, x2, kh, kw, sh, pt, pl, oh, ow, cout, math="bf16x3")
        if not K._halo_ok(mode, args):
            continue
        C = c1 + c2
        wt = torch.randn(kh, kw, C, cout, device=dev, generator=g) / (kh * kw * C) ** 0.5
        wn, wd = K.filter_to_native(wt), K.filter_to_dgrad(wt)
        K.filter_split(wn, torch.empty_like(wn))
        K.filter_split(wd, torch.empty_like(wd))
        y = torch.empty(n, oh, ow, cout, device=dev)
        dy = torch.randn(n, oh, ow, cout, device=dev, generator=g)
        dx1, dx2 = torch.empty_like(x1), (torch.empty_like(x2) if c2 else None)

        def run():
            if mode == "fwd":
                K.conv2d_fwd(args, wn, None, y)
            else:
                K.conv2d_dgrad(args, dy, wd, dx1, dx2)

        def timed(t):
            args.tile = t
            run()
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
            return best

        cur = K._TILE_CACHE[key]
        t_cur = timed(cur)
        times = {t: timed(t) for t in halo}
        best = min(times, key=times.get)
        pick = best if times[best] < t_cur * (1 - a.margin) else cur
        K._TILE_CACHE[key] = pick
        row = {"key": list(key), "table": K.schedule_desc(m, cur), "table_ms": round(t_cur, 4),
               "best_halo": K.schedule_desc(m, best), "halo_ms": round(times[best], 4),
               "picked": K.schedule_desc(m, pick)}
        report.append(row)
        print(f"{mode:5s} {n}x{h}x{w} c{c1}+{c2} -> {cout}: {row['table']} {t_cur:.3f} ms | "
              f"{row['best_halo']} {times[best]:.3f} ms -> {row['picked']}", flush=True)
        del x1, x2, wt, wn, wd, y, dy, dx1, dx2
        torch.cuda.empty_cache()
    out = a.out or table
    K.save_tile_cache(out)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "halo_tune.json"), "w") as f:
        json.dump(report, f, indent=1)
    print("written", out, flush=True)


if __name__ == "__main__":
    main()
