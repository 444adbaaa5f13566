"""A/B timing of the wide 1x1 bf16x3 kernel on the ff_effnet 448x448 b32 shapes.

    python tools/wide_ab.py            # wide1x1_kernel where eligible
    PLD_NO_WIDE=1 python tools/wide_ab.py   # the im2col tiles (autotuned)
Prints one line per (mode, M, K, N): kernel name, median us, GB/s of algorithmic bytes.
"""
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pldepth_amd import kernels as K  # noqa: E402

SHAPES = [  # (rows, K, N) of the GEMM
    (100352, 40, 240), (100352, 40, 144), (25088, 80, 240), (25088, 80, 480),
    (25088, 112, 480), (25088, 112, 672), (6272, 112, 672), (6272, 128, 1152),
]
if os.environ.get("WIDE_AB_BIG"):  # asymptotic rates (8x the rows)
    SHAPES = [(8 * r, k, n) for r, k, n in SHAPES[2:]]
if os.environ.get("WIDE_AB_ONLY"):  # one shape (PMC passes)
    SHAPES = [SHAPES[int(os.environ["WIDE_AB_ONLY"])]]
REPS = int(os.environ.get("WIDE_AB_REPS", "30"))


def timed(fn, reps=None):
    reps = reps or REPS
    for _ in range(3):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(reps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    t = sorted(a.elapsed_time(b) for a, b in ev)
    return 1e3 * t[len(t) // 2]


def main():
    dev = torch.device("cuda:0")
    lib = K.lib()
    for rows, k, n in SHAPES:
        h = 56 if rows % (56 * 56) == 0 else (28 if rows % (28 * 28) == 0 else 14)
        b = rows // (h * h)
        x = torch.randn(b, h, h, k, device=dev)
        wt = torch.randn(1, 1, k, n, device=dev) / k ** 0.5
        wn = K.filter_to_native(wt)
        y = torch.empty(b, h, h, n, device=dev)
        args = K.conv_args(x, None, 1, 1, 1, 0, 0, h, h, n, math="bf16x3")
        name = lib.pld_conv_kernel_name(C.byref(args), 0).decode()
        us = timed(lambda: K.conv2d_fwd(args, wn, None, y))
        m = torch.empty(n, device=dev)
        i = torch.empty(n, device=dev)
        us_st = timed(lambda: K.conv2d_fwd_bn_stats(args, wn, None, y, m, i))
        gb = 4.0 * rows * (k + n) / 1e9
        print(f"fwd   {rows:7d} {k:4d} {n:5d} {name:24s} {us:8.1f} us {gb / us * 1e6:7.0f} GB/s"
              f"   +stats {us_st:8.1f} us", flush=True)


if __name__ == "__main__":
    main()
