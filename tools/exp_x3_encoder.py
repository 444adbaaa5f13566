"""Forward-activation error vs the fp64 oracle for a conv math policy at several input sizes.

    python tools/exp_x3_encoder.py --sizes 64 224 448 --batch 2 --policy bf16x3 mixed
"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp(min=1e-30))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", type=int, nargs="+", default=[64, 224, 448])
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--policy", nargs="+", default=["bf16x3", "mixed"])
    a = ap.parse_args()
    from oracle import effnet as OE
    from pldepth_amd import kernels as K
    from pldepth_amd.models.effnet_ff import EffNetFF
    torch.set_num_threads(16)
    taps_names = ["stem_activation", "block2a_output", "block3a_expand_activation",
                  "block4a_output", "block5c_output", "block6a_expand_activation",
                  "block7a_output", "top_activation"]
    for H in a.sizes:
        B = a.batch
        rng = np.random.default_rng(0)
        x = rng.random((B, H, H, 3)).astype(np.float32)
        ref = None
        for pol in a.policy:
            eng = EffNetFF((H, H, 3), B, seed=0, conv_math=pol)
            eng.drop_connect = False
            if ref is None:
                w = eng.get_weights()
                P = {k: torch.tensor(v, dtype=torch.float64) for k, v in w.items()}
                taps = {}
                with torch.no_grad():
                    pred_ref = OE.forward(P, torch.tensor(x, dtype=torch.float64), taps=taps)
                ref = (taps, pred_ref)
            eng.act["input"].copy_(torch.from_numpy(x))
            pred = eng.forward(training=True)
            torch.cuda.synchronize()
            taps, pred_ref = ref
            errs = {n: rel(eng.act[n], taps[n].permute(0, 2, 3, 1)) for n in taps_names
                    if n in eng.act}
            errs["pred"] = rel(pred, pred_ref)
            print(f"H={H} B={B} policy={pol}: " +
                  " ".join(f"{k}={v:.2e}" for k, v in errs.items()), flush=True)
            del eng
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
