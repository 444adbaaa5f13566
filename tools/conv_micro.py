"""Time one implicit-GEMM conv shape in isolation (for rocprofv3 counter passes and tile sweeps).

    python tools/conv_micro.py --mode fwd --n 32 --h 28 --w 28 --c1 672 --c2 672 --k 3 \
        --cout 240 [--math bf16x3] [--tile -1] [--iters 20]

Prints per-launch time and TF/s (HIP events on the current stream).
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="fwd", choices=["fwd", "dgrad", "wgrad"])
    ap.add_argument("--n", type=int, default=32)
    ap.add_argument("--h", type=int, default=28)
    ap.add_argument("--w", type=int, default=28)
    ap.add_argument("--c1", type=int, default=672)
    ap.add_argument("--c2", type=int, default=0)
    ap.add_argument("--k", type=int, default=3)
    ap.add_argument("--cout", type=int, default=240)
    ap.add_argument("--math", default="bf16x3")
    ap.add_argument("--tile", type=int, default=-1, help="-1 = autotune")
    ap.add_argument("--sched", default="", help="schedule by name (pld_conv_schedule_desc), "
                    "e.g. x3split/128x128; overrides --tile")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--presplit", type=int, default=1)
    ap.add_argument("--acc", type=int, default=0, help="accumulate into the destination")
    a = ap.parse_args()
    from pldepth_amd import kernels as K
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    x1 = torch.randn(a.n, a.h, a.w, a.c1, device=dev, generator=g)
    x2 = torch.randn(a.n, a.h, a.w, a.c2, device=dev, generator=g) if a.c2 else None
    C = a.c1 + a.c2
    w = torch.randn(a.k, a.k, C, a.cout, device=dev, generator=g) / (a.k * a.k * C) ** 0.5
    pt = (a.k - 1) // 2
    args = K.conv_args(x1, x2, a.k, a.k, 1, pt, pt, a.h, a.w, a.cout, math=a.math)
    args.tile = a.tile
    if a.sched:
        idx = K._schedule_index(K.MATH[a.math], a.sched)
        assert idx is not None, f"no schedule named {a.sched}"
        args.tile = idx
    wn, wd = K.filter_to_native(w), K.filter_to_dgrad(w)
    if a.presplit and a.math == "bf16x3":
        if C % 8 == 0:
            K.filter_split(wn, torch.empty_like(wn))
        if a.cout % 8 == 0:
            K.filter_split(wd, torch.empty_like(wd))
    y = torch.empty(a.n, a.h, a.w, a.cout, device=dev)
    dy = torch.randn_like(y)
    dx1, dx2 = torch.empty_like(x1), (torch.empty_like(x2) if x2 is not None else None)
    dw = torch.empty_like(w)
    run = {"fwd": lambda: K.conv2d_fwd(args, wn, None, y, accumulate=bool(a.acc)),
           "dgrad": lambda: K.conv2d_dgrad(args, dy, wd, dx1, dx2, acc1=bool(a.acc)),
           "wgrad": lambda: K.conv2d_wgrad(args, dy, dw)}[a.mode]
    run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        run()
    e1.record()
    e1.synchronize()
    ms = e0.elapsed_time(e1) / a.iters
    fl = 2.0 * a.n * a.h * a.w * a.cout * a.k * a.k * C
    print(f"{a.mode} n{a.n} {a.h}x{a.w} c{a.c1}+{a.c2} k{a.k} cout{a.cout} {a.math} "
          f"tile={args.tile} {a.sched}: {ms:.3f} ms  {fl / ms / 1e9:.1f} TF/s")


if __name__ == "__main__":
    main()
