"""Time pld_se_bwd_bn_full (SE squeeze backward with the block BN's reductions, the excitation
FC backward, the BN backward apply) on MBConv block shapes at batch 32 (HIP events).

    python tools/se_micro.py [--iters 20]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (block, hw side, channels, squeeze channels) of EfficientNetB0 at 448x448
SHAPES = [("1a", 224, 32, 8), ("2a", 112, 96, 4), ("2b", 112, 144, 6), ("3b", 56, 240, 10),
          ("5b", 28, 672, 28), ("6b", 14, 1152, 48)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--n", type=int, default=32)
    a = ap.parse_args()
    from pldepth_amd import kernels as K
    torch.cuda.set_device(0)
    g = torch.Generator(device="cuda").manual_seed(0)
    for name, hw, c, cse in SHAPES:
        n = a.n
        r = lambda *s: torch.randn(*s, device="cuda", generator=g)
        x, dy = r(n, hw, hw, c), r(n, hw, hw, c)
        bn = (r(c) * 0.1, torch.rand(c, device="cuda") + 0.5, r(c), r(c))
        w1, w2 = r(c, cse) * 0.1, r(cse, c) * 0.1
        z1, gate = r(n, cse), torch.rand(n, c, device="cuda")
        addn, dx = torch.empty(n, c, device="cuda"), torch.empty_like(x)
        dg, db = torch.empty(c, device="cuda"), torch.empty(c, device="cuda")
        run = lambda: K.se_bwd_bn_full(dy, x, bn, w1, w2, z1, gate, addn, dx, dg, db)
        run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            run()
        e1.record()
        e1.synchronize()
        ms = e0.elapsed_time(e1) / a.iters
        gb = x.numel() * 4 * 5 / 1e9  # squeeze reads (x, dy); apply reads (x, dy), writes dx
        print(f"{name} {n}x{hw}x{hw}x{c}: {ms * 1e3:.1f} us  {gb / ms * 1e3:.0f} GB/s (5 passes of "
              f"4 B/elem)")


if __name__ == "__main__":
    main()
