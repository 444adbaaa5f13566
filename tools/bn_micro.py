"""BN reduction/apply microbenchmark (GPU box): times pld_bn_stats, pld_bn_bwd (reduce + apply)
and pld_bn_apply on one NHWC shape with HIP events; prints achieved HBM GB/s per call.

    python tools/bn_micro.py --rows 1605632 --c 96 [--iters 20]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pldepth_amd import kernels as K  # noqa: E402


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1605632)
    ap.add_argument("--c", type=int, default=96)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--act", default="swish")
    a = ap.parse_args()
    d = torch.device("cuda")
    r, c = a.rows, a.c
    x = torch.randn(r, c, device=d)
    dy = torch.randn(r, c, device=d)
    dx = torch.empty_like(x)
    y = torch.empty_like(x)
    mean, inv = torch.zeros(c, device=d), torch.ones(c, device=d)
    g, b = torch.ones(c, device=d), torch.zeros(c, device=d)
    dg, db = torch.empty(c, device=d), torch.empty(c, device=d)
    nb = r * c * 4
    t_st = timeit(lambda: K.bn_stats(x, r, c, mean, inv), a.iters)
    t_bw = timeit(lambda: K.bn_bwd(x, dy, r, c, mean, inv, g, b, a.act, dx, dg, db), a.iters)
    t_ap = timeit(lambda: K.bn_apply(x, r, c, mean, inv, g, b, a.act, y), a.iters)
    tag = f"blocks={os.environ.get('PLD_RED_BLOCKS', '2048')} ru={os.environ.get('PLD_RED_RU', '4')}"
    print(f"rows={r} c={c} {tag}: stats {t_st * 1e3:.1f} us ({nb / t_st / 1e6:.0f} GB/s, "
          f"incl. finalize) | bwd {t_bw * 1e3:.1f} us ({5 * nb / t_bw / 1e6:.0f} GB/s reduce+apply)"
          f" | apply {t_ap * 1e3:.1f} us ({2 * nb / t_ap / 1e6:.0f} GB/s)", flush=True)


if __name__ == "__main__":
    main()
