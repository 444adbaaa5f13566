"""How much does the cfg1 (224x224, batch 2) gradient parity move under ulp-level rounding changes?

Runs the cfg1 trainer step once on the GPU (as tests/test_configs_gpu.py::test_cfg1_trainer_step_224)
for its weights, rankings and drop-connect scales, then the fp32 restatement of the step several
times with the input image perturbed by one fp32 ulp in random directions (stand-ins for another
fp32 summation order in the stem), and prints each run's per-tensor error vs fp64 for the
tensors the test flags plus the global rel-L2: the spread is what any fp32 implementation can land
on, i.e. how much of a per-tensor bar at 4x one fp32 run's error is rounding luck.

    python tools/exp_cfg1_sensitivity.py [--runs 4] [--out FILE]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

WATCH = ["dec_bn3/beta", "dec_conv3/kernel", "dec_bn2/gamma", "dec_bn0/gamma", "dec_conv4/kernel"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=4)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    from oracle import effnet as OE
    from oracle import listmle as LM
    from pldepth_amd.trainer import ReplicaTrainer
    from tests.test_configs_gpu import _residual_drop_blocks
    torch.cuda.set_device(0)
    cuda = torch.device("cuda", 0)
    B, H, L, R, lr = 2, 224, 2, 100, 0.01
    tr = ReplicaTrainer((H, H, 3), B, L, R, 1, seed=0)
    eng = tr.engine
    rng = np.random.default_rng(9)
    x = rng.random((B, H, H, 3)).astype(np.float32)
    yy, xx = np.meshgrid(np.linspace(0, 1, H), np.linspace(0, 1, H), indexing="ij")
    gt = np.stack([np.round(255 * (0.5 + 0.3 * np.sin((3 + b) * yy) * np.cos(2 * xx))) / 255
                   for b in range(B)]).astype(np.float32)
    mask = (rng.random((B, H, H)) < 0.9).astype(np.float32)
    weights = eng.get_weights()
    tr.set_batch(torch.from_numpy(x).to(cuda), torch.from_numpy(gt).to(cuda),
                 torch.from_numpy(mask).to(cuda))
    tr.step_eager(lr)
    tr.synchronize()
    y = tr.y_true.cpu().numpy()
    drop = {blk["name"]: torch.tensor(blk["drop"].cpu().numpy(), dtype=torch.float64)
            for li, blk in _residual_drop_blocks(eng)}
    hip = {k: eng.grads[k].detach().cpu().double() for k in OE.trainable_names(weights)}
    torch.set_num_threads(16)
    P = {k: torch.tensor(v, dtype=torch.float64) for k, v in weights.items()}
    x64 = torch.tensor(x, dtype=torch.float64)
    with torch.no_grad():
        pred_ref = OE.forward(P, x64, drop_scales=drop)
    _, dpred_ref = LM.hourglass_nll(y, pred_ref.numpy(), B, L)
    g64, _ = OE.train_step_grads(P, x64, torch.tensor(dpred_ref), drop_scales=drop)
    keys = [k for k in g64 if float(g64[k].abs().max()) > 0]
    ref = torch.cat([g64[k].double().flatten() for k in keys])

    def report(tag, g):
        e = {k: float((g[k].double() - g64[k]).abs().max() / g64[k].abs().max()) for k in keys}
        flat = torch.cat([g[k].double().flatten() for k in keys])
        out = {"global_rel_l2": float((flat - ref).norm() / ref.norm()),
               "watch": {k: e[k] for k in WATCH if k in e}}
        print(tag, json.dumps(out), flush=True)
        return out

    res = {"hip": report("hip", hip)}
    P32 = {k: torch.tensor(v, dtype=torch.float32) for k, v in weights.items()}
    d32 = {k: v.float() for k, v in drop.items()}
    g = torch.Generator().manual_seed(1)
    for r in range(a.runs):
        xp = torch.tensor(x)
        if r > 0:  # one ulp up or down per element
            sgn = torch.randint(0, 2, xp.shape, generator=g) * 2 - 1
            xp = torch.nextafter(xp, xp + sgn.float())
        g32, _ = OE.train_step_grads(P32, xp, torch.tensor(dpred_ref).float(), drop_scales=d32)
        res[f"fp32_run{r}"] = report(f"fp32 run {r} ({'input as is' if r == 0 else 'input +-1 ulp'})",
                                     g32)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
