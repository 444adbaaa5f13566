"""Time every conv schedule of one shape from a replayed hipGraph (no host launch gaps).

    python tools/sched_sweep.py --mode dgrad --n 32 --h 14 --w 14 --c1 1152 --k 1 --cout 192

For each schedule index the shape takes (kernels._schedules), 10 launches are captured into a
graph that is replayed 5 times; prints us per launch, TF/s and algorithmic GB/s, fastest first.
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def sweep(mode, n, h, w, c1, c2, k, cout, math="bf16x3", reps=10, replays=5, scheds=None,
          stride=1, pad=None):
    from pldepth_amd import kernels as K
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    x1 = torch.randn(n, h, w, c1, device=dev, generator=g)
    x2 = torch.randn(n, h, w, c2, device=dev, generator=g) if c2 else None
    C = c1 + c2
    wt = torch.randn(k, k, C, cout, device=dev, generator=g) / (k * k * C) ** 0.5
    pt = (k - 1) // 2 if pad is None else pad
    oh, ow = (h - 1) // stride + 1, (w - 1) // stride + 1
    wn, wd = K.filter_to_native(wt), K.filter_to_dgrad(wt)
    if math == "bf16x3":
        if C % 8 == 0:
            K.filter_split(wn, torch.empty_like(wn))
        if cout % 8 == 0:
            K.filter_split(wd, torch.empty_like(wd))
    y = torch.empty(n, oh, ow, cout, device=dev)
    dy = torch.randn_like(y)
    dx1, dx2 = torch.empty_like(x1), (torch.empty_like(x2) if x2 is not None else None)
    dw = torch.empty_like(wt)
    base = K.conv_args(x1, x2, k, k, stride, pt, pt, oh, ow, cout, math=math)
    fl = 2.0 * n * oh * ow * cout * k * k * C
    by = 4.0 * (n * h * w * C + n * oh * ow * cout + k * k * C * cout)
    out = []
    st = torch.cuda.Stream()
    for t in (scheds if scheds is not None else K._schedules(mode, base.math, base)):
        args = K.conv_args(x1, x2, k, k, stride, pt, pt, oh, ow, cout, math=math)
        args.tile = t
        run = {"fwd": lambda: K.conv2d_fwd(args, wn, None, y),
               "dgrad": lambda: K.conv2d_dgrad(args, dy, wd, dx1, dx2),
               "wgrad": lambda: K.conv2d_wgrad(args, dy, dw)}[mode]
        with torch.cuda.stream(st):
            run()  # sizes the workspaces outside the capture
            st.synchronize()
            gr = K.Graph().capture(lambda: [run() for _ in range(reps)])
            gr.launch()
            st.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(replays):
                gr.launch()
            e1.record(st)
            e1.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / (reps * replays)
        out.append((us, t, K.schedule_desc(args.math, t), K.conv_kernel_name(args, mode)))
        del gr
    out.sort()
    return out, fl, by


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="fwd", choices=["fwd", "dgrad", "wgrad"])
    ap.add_argument("--n", type=int, default=32)
    ap.add_argument("--h", type=int, default=14)
    ap.add_argument("--w", type=int, default=14)
    ap.add_argument("--c1", type=int, default=192)
    ap.add_argument("--c2", type=int, default=0)
    ap.add_argument("--k", type=int, default=1)
    ap.add_argument("--cout", type=int, default=1152)
    ap.add_argument("--math", default="bf16x3")
    ap.add_argument("--stride", type=int, default=1)
    ap.add_argument("--pad", type=int, default=None, help="top/left padding (default (k-1)/2)")
    ap.add_argument("--top", type=int, default=8)
    ap.add_argument("--sched", type=int, nargs="*", default=None,
                    help="only these schedule indices (e.g. for a rocprofv3 counter pass)")
    a = ap.parse_args()
    torch.cuda.set_device(0)
    res, fl, by = sweep(a.mode, a.n, a.h, a.w, a.c1, a.c2, a.k, a.cout, a.math,
                        scheds=a.sched, stride=a.stride, pad=a.pad)
    print(f"{a.mode} n{a.n} {a.h}x{a.w} c{a.c1}+{a.c2} k{a.k} cout{a.cout} {a.math}: "
          f"{fl / 1e9:.2f} GFLOP, {by / 1e6:.1f} MB algorithmic")
    for us, t, desc, kname in res[:a.top]:
        print(f"  {us:8.2f} us  {fl / us / 1e6:6.1f} TF/s  {by / us / 1e3:6.0f} GB/s  "
              f"[{t}] {desc} {kname}")


if __name__ == "__main__":
    main()
