"""Debug the bf16x3 tile-stream schedules: fwd of small convs per stream schedule against fp64,
printing which output rows / columns go wrong.

    python tools/debug_stream.py
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def ref_conv(x, w, k):
    p = (k - 1) // 2
    y = torch.nn.functional.conv2d(x.permute(0, 3, 1, 2).double(),
                                   w.permute(3, 2, 0, 1).double(), padding=p)
    return y.permute(0, 2, 3, 1)


def main():
    from pldepth_amd import _lib
    from pldepth_amd import kernels as K
    torch.cuda.set_device(0)
    lib = _lib.lib()
    m = K.MATH["bf16x3"]
    cases = [(1, 8, 8, 32, 1, 32), (2, 14, 14, 128, 3, 64), (2, 14, 14, 128, 1, 64),
             (4, 32, 32, 64, 1, 64)]
    for (n, h, w, c, k, cout) in cases:
        torch.manual_seed(0)
        x = torch.randn(n, h, w, c, device="cuda")
        wt = torch.randn(k, k, c, cout, device="cuda") / (k * k * c) ** 0.5
        wn = K.filter_to_native(wt)
        ref = ref_conv(x.cpu(), wt.cpu(), k)
        for t in range(lib.pld_conv_num_schedules(m)):
            if lib.pld_conv_schedule_class(m, t) not in (0, 5):
                continue
            args = K.conv_args(x, None, k, k, 1, (k - 1) // 2, (k - 1) // 2, h, w, cout,
                               math="bf16x3")
            args.tile = t
            y = torch.zeros(n, h, w, cout, device="cuda")
            K.conv2d_fwd(args, wn, None, y)
            torch.cuda.synchronize()
            d = (y.double().cpu() - ref).abs()
            err = float(d.max() / ref.abs().max())
            if err > 1e-4:
                bad = (d.reshape(-1, cout) > 1e-3 * float(ref.abs().max()))
                rows = bad.any(1).nonzero().flatten().tolist()
                cols = bad.any(0).nonzero().flatten().tolist()
                print(f"case {(n, h, w, c, k, cout)} sched {t} {K.schedule_desc(m, t)}: err "
                      f"{err:.3e} bad rows {len(rows)}/{n * h * w} first {rows[:12]} cols "
                      f"{cols[:8]}..{len(cols)}", flush=True)
            else:
                print(f"case {(n, h, w, c, k, cout)} sched {t} {K.schedule_desc(m, t)}: ok",
                      flush=True)


if __name__ == "__main__":
    main()
