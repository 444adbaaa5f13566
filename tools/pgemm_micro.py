"""Time pld_pgemm_bn_act / _bn_bwd against the unfused pairs they replace at the ff_effnet
448x448 batch-32 shapes (project convs over BN+swish+gate, expand dgrads over the BN backward).

    python tools/pgemm_micro.py [--iters 20]
"""
import argparse
import os
import sys

import torch  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# (name, images, hw, K = cexp, N): project convs (fwd) and expand dgrads (bwd)
SHAPES = [("1a_proj", 32, 224 * 224, 32, 16), ("2a_proj", 32, 112 * 112, 96, 24),
          ("2b_proj", 32, 112 * 112, 144, 24), ("3a_proj", 32, 56 * 56, 144, 40),
          ("3b_proj", 32, 56 * 56, 240, 40),
          ("2a_exdg", 32, 224 * 224, 96, 16), ("2b_exdg", 32, 112 * 112, 144, 24),
          ("3a_exdg", 32, 112 * 112, 144, 24), ("3b_exdg", 32, 56 * 56, 240, 40),
          ("4a_exdg", 32, 56 * 56, 240, 40)]


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from pldepth_amd import kernels as K
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    for name, n, hw, k, nn in SHAPES:
        rows = n * hw
        x = torch.randn(n, hw, 1, k, device=dev, generator=g)
        bn = [torch.rand(k, device=dev, generator=g) + 0.5 for _ in range(4)]
        y = torch.empty(n, hw, 1, nn, device=dev)
        if name.endswith("proj"):
            gate = torch.rand(n, k, device=dev, generator=g)
            w = torch.randn(nn, k, device=dev, generator=g)
            fused = lambda: K.pgemm_bn_act(x, rows, k, *bn, "swish", w, nn, y, gate=gate, hw=hw)
            a_ = torch.empty_like(x)
            args = K.conv_args(a_, None, 1, 1, 1, 0, 0, hw, 1, nn, math="bf16x3")
            wn = w.view(nn, 1, 1, k).contiguous()

            def unfused():
                K.bn_apply(x, rows, k, *bn, "swish", a_, gate=gate, hw=hw)
                K.conv2d_fwd(args, wn, None, y)
            by = 4.0 * rows * (k + nn)
        else:
            dy = torch.randn_like(x)
            k12 = torch.randn(2 * k, device=dev, generator=g) * 0.01
            w = torch.randn(nn, k, device=dev, generator=g)
            dg, db = torch.empty(k, device=dev), torch.empty(k, device=dev)
            fused = lambda: K.pgemm_bn_bwd(x, dy, rows, k, *bn, "swish", k12, w, nn, y)
            gpe = torch.empty_like(x)
            args = K.conv_args(y, None, 1, 1, 1, 0, 0, hw, 1, k, math="bf16x3")
            wd = w.view(nn, 1, 1, k).contiguous()

            def unfused():
                K.bn_bwd(x, dy, rows, k, *bn, "swish", gpe, dg, db)
                K.conv2d_dgrad(args, gpe, wd, y)
            by = 4.0 * rows * (2 * k + nn)
        tf = timeit(fused, a.iters)
        tu = timeit(unfused, a.iters)
        print(f"{name:8s} rows {rows:8d} K {k:3d} N {nn:2d}: fused {tf * 1e3:7.1f} us "
              f"({by / tf / 1e9:5.2f} TB/s)   unfused {tu * 1e3:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
