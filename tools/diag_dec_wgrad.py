"""Where does a decoder weight gradient's error come from? (dec_conv4/kernel at
batch 32 is 1.8e-3 from fp64 against the fp32 restatement's 9.3e-4.)

Runs the bench's ff_effnet step (448x448, batch 32, 'auto' policy, the given schedule table)
on the GPU, then recomputes every decoder conv's dW in fp64 on the CPU from the GPU's OWN
operands (the conv input and the pre-BN output gradient the HIP backward used). The printed
`arith` error is the wgrad kernel's arithmetic alone; the rest of the HIP-vs-oracle error comes
from the operands (forward activations and the upstream backward).

    python tools/diag_dec_wgrad.py [--schedules PATH] [--math bf16x3|fp32]
"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--schedules", default="")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--size", type=int, default=448)
    a = ap.parse_args()
    from pldepth_amd import kernels as K
    from pldepth_amd.models.effnet_ff import EffNetFF
    if a.schedules:
        print("schedule entries:", K.use_schedule_table(a.schedules))
    torch.cuda.set_device(0)
    B, H, R, L = a.batch, a.size, 100, 5
    rng = np.random.default_rng(32)
    x = rng.random((B, H, H, 3)).astype(np.float32)
    eng = EffNetFF((H, H, 3), B, seed=0, conv_math="auto")
    eng.drop_connect = False
    # decoder pre-BN gradients live in the side-stream slot "dec" (one buffer per shape, never
    # reused by the encoder backward)
    assert eng.overlap_wgrad
    eng.act["input"].copy_(torch.from_numpy(x))
    pred = eng.forward(training=True)
    idx = rng.integers(0, H * H, (B, R, L))
    lab = -np.sort(-(rng.permutation(B * R * L).reshape(B, R, L) / (B * R * L)), axis=-1)
    y = np.ascontiguousarray(np.stack([idx.astype(np.float32), lab.astype(np.float32)], -1))
    _, dpred, _ = K.listmle_fwd_bwd(pred, torch.from_numpy(y).cuda(), B, R, L)
    eng.backward(dpred)
    torch.cuda.synchronize()
    A = eng.act
    h = H
    torch.set_num_threads(16)
    for i in range(len(eng.dec) - 1, -1, -1):
        conv, bn, skip = eng.dec[i]
        h //= 2
        if i == 0:
            xs = [A["top_activation"]]
        else:
            xs = [A[f"dec{i - 1}_up"]] + ([A[eng.dec[i - 1][2]]] if eng.dec[i - 1][2] else [])
        xin = torch.cat([t.double().cpu() for t in xs], dim=3).permute(0, 3, 1, 2)
        gpre = eng._gpre_buf(A[f"dec{i}_pre"].shape, "dec").double().cpu().permute(0, 3, 1, 2)
        dw64 = torch.nn.grad.conv2d_weight(xin, (conv.cout, xin.shape[1], 3, 3), gpre,
                                           padding=1)  # [cout][cin][ky][kx]
        hip = conv.dw.double().cpu()  # HWIO
        ref = dw64.permute(2, 3, 1, 0)
        e = float((hip - ref).abs().max() / ref.abs().max())
        # cancellation: sum |x dy| over the products vs |sum x dy| (max over the outputs)
        absx = torch.nn.grad.conv2d_weight(xin.abs(), (conv.cout, xin.shape[1], 3, 3),
                                           gpre.abs(), padding=1)
        canc = float(absx.max() / dw64.abs().max())
        print(f"dec_conv{i}: {tuple(xin.shape)} -> {conv.cout}: arith rel err {e:.3e}, "
              f"sum|x dy| / max|dW| {canc:.1f}", flush=True)


if __name__ == "__main__":
    main()
