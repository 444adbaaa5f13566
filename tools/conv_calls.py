"""Every conv call of one eager ff_effnet (or ff_redweb) training step: shape, mode, the kernel
and schedule it ran, HIP-event time, algorithmic TF/s and TB/s. Sorted by time; totals per
kernel. For finding which launches a kernel family's time is made of.

    python tools/conv_calls.py [--model ff_effnet] [--batch 32] [--size 448] [--kernel conv_x3_kernel]
"""
import argparse
import collections
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="ff_effnet")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--size", type=int, default=448)
    ap.add_argument("--kernel", default="", help="list only calls of this kernel")
    a = ap.parse_args()
    import bench
    from pldepth_amd import kernels as K
    from pldepth_amd._lib import lib
    torch.cuda.set_device(0)
    K.use_schedule_table()
    tr, _ = bench.run_config(a.model, a.size, a.batch, 5, 100, "info", 1, 1, 0, 1, None,
                             graph=False)
    st = tr.stream
    mode_of = {"conv2d_fwd": 0, "conv2d_dgrad": 1, "conv2d_wgrad": 2, "conv2d_fwd_bn_stats": 0}
    orig = {n: getattr(K, n) for n in mode_of}
    recs = []

    def wrap(name):
        fn = orig[name]

        def w(args, *rest, **kw):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            r = fn(args, *rest, **kw)
            e1.record(st)
            tile = getattr(args, "_used_tile", args.tile)
            saved, args.tile = args.tile, tile
            kname = lib().pld_conv_kernel_name(ctypes.byref(args), mode_of[name]).decode()
            args.tile = saved
            C = args.c1 + args.c2
            fl = 2.0 * args.n * args.oh * args.ow * args.cout * args.kh * args.kw * C
            by = 4.0 * (args.n * args.h * args.w * C + args.n * args.oh * args.ow * args.cout
                        + args.kh * args.kw * C * args.cout)
            shape = (f"{['fwd', 'dgrad', 'wgrad'][mode_of[name]]} {args.kh}x{args.kw}/{args.sh} "
                     f"{args.h}x{args.w} {args.c1}+{args.c2}->{args.cout}")
            sched = K.schedule_desc(args.math, tile) if tile >= 0 else str(tile)
            recs.append((kname.split("(")[0], shape, sched, fl, by, e0, e1))
            return r
        return w

    for n in mode_of:
        setattr(K, n, wrap(n))
    try:
        tr.step_eager(0.01)
        torch.cuda.synchronize()
    finally:
        for n, f in orig.items():
            setattr(K, n, f)
    rows = [(k, s, sc, fl, by, e0.elapsed_time(e1) * 1e-3) for k, s, sc, fl, by, e0, e1 in recs]
    tot = collections.defaultdict(lambda: [0, 0.0])
    for k, s, sc, fl, by, t in rows:
        tot[k][0] += 1
        tot[k][1] += t
    for k, (n, t) in sorted(tot.items(), key=lambda kv: -kv[1][1]):
        print(f"{t * 1e3:8.3f} ms {n:3d} x  {k}")
    print()
    for k, s, sc, fl, by, t in sorted(rows, key=lambda r: -r[5]):
        if a.kernel and a.kernel not in k:
            continue
        print(f"{t * 1e6:8.1f} us {fl / t / 1e12:6.1f} TF/s {by / t / 1e12:5.2f} TB/s  "
              f"{s:34s} {sc:24s} {k[-60:]}")


if __name__ == "__main__":
    main()
