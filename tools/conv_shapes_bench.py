"""Time the decoder conv shapes of the ff_effnet step at batch 32 (448x448) in isolation:
autotuned schedule, per-launch ms, TF/s and the kernel each call runs.

    python tools/conv_shapes_bench.py [--iters 10] [--only fwd,dgrad,wgrad]
"""
import argparse
import ctypes as C
import os
import sys

import torch  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# (name, h, w, c1, c2, cout): the five 3x3 decoder convs (pl_hourglass.py:59-91) at 448x448
SHAPES = [("dec0", 14, 14, 1280, 0, 672), ("dec1", 28, 28, 672, 672, 240),
          ("dec2", 56, 56, 240, 240, 144), ("dec3", 112, 112, 144, 144, 32),
          ("dec4", 224, 224, 32, 0, 32)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--n", type=int, default=32)
    ap.add_argument("--only", default="fwd,dgrad,wgrad")
    a = ap.parse_args()
    from pldepth_amd import kernels as K
    from pldepth_amd._lib import lib
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    total = 0.0
    for name, h, w, c1, c2, cout in SHAPES:
        x1 = torch.randn(a.n, h, w, c1, device=dev, generator=g)
        x2 = torch.randn(a.n, h, w, c2, device=dev, generator=g) if c2 else None
        Cin = c1 + c2
        wt = torch.randn(3, 3, Cin, cout, device=dev, generator=g) / (9 * Cin) ** 0.5
        wn, wd = K.filter_to_native(wt), K.filter_to_dgrad(wt)
        K.filter_split(wn, torch.empty_like(wn))
        if cout % 8 == 0:
            K.filter_split(wd, torch.empty_like(wd))
        y = torch.empty(a.n, h, w, cout, device=dev)
        dy = torch.randn_like(y)
        dx1 = torch.empty_like(x1)
        dx2 = torch.empty_like(x2) if x2 is not None else None
        dw = torch.empty_like(wt)
        for mode in a.only.split(","):
            args = K.conv_args(x1, x2, 3, 3, 1, 1, 1, h, w, cout, math="bf16x3")
            run = {"fwd": lambda: K.conv2d_fwd(args, wn, None, y),
                   "dgrad": lambda: K.conv2d_dgrad(args, dy, wd, dx1, dx2),
                   "wgrad": lambda: K.conv2d_wgrad(args, dy, dw)}[mode]
            run()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                run()
            e1.record()
            e1.synchronize()
            ms = e0.elapsed_time(e1) / a.iters
            fl = 2.0 * a.n * h * w * cout * 9 * Cin
            saved = args.tile
            args.tile = getattr(args, "_used_tile", saved)
            kn = lib().pld_conv_kernel_name(C.byref(args), {"fwd": 0, "dgrad": 1,
                                                            "wgrad": 2}[mode]).decode()
            sched = args.tile
            args.tile = saved
            total += ms
            print(f"{name} {mode:5s} {ms:7.3f} ms {fl / ms / 1e9:7.1f} TF/s  sched {sched:3d} "
                  f"{kn}", flush=True)
    print(f"total {total:.3f} ms")


if __name__ == "__main__":
    main()
