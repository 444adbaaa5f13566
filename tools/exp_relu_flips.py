"""Why does the cfg1 dec_bn3/beta gradient swing with the stem's rounding? Counts the decoder
ReLU sign flips (pre-activation z = BN(conv) on opposite sides of 0) between the HIP step and
the fp64 oracle, and between the fp32 restatement and fp64, per decoder stage, beside each BN
beta gradient's per-channel error: a pixel whose z crosses 0 passes its whole upstream gradient in
one realization and none in the other.

    python tools/exp_relu_flips.py [--out FILE]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    from oracle import effnet as OE
    from oracle import listmle as LM
    from pldepth_amd import kernels as K
    from pldepth_amd.trainer import ReplicaTrainer
    from tests.test_configs_gpu import _residual_drop_blocks
    K.AUTOTUNE = False  # the built-in schedules, as the test's fixed_schedules
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
    torch.set_num_threads(16)
    res = {}
    zs = {}
    for tag, dt in (("fp64", torch.float64), ("fp32", torch.float32)):
        P = {k: torch.tensor(v, dtype=dt) for k, v in weights.items()}
        taps = {}
        with torch.no_grad():
            pred = OE.forward(P, torch.tensor(x, dtype=dt),
                              drop_scales={k: v.to(dt) for k, v in drop.items()}, taps=taps)
            z = {}
            xin = taps["top_activation"]
            for i, (name, cout, skip) in enumerate(OE.DECODER):
                c = OE.conv_same(xin, P[name + "/kernel"], P[name + "/bias"])
                z[i] = OE.bn_train(c, P[f"dec_bn{i}/gamma"], P[f"dec_bn{i}/beta"])
                xin = taps[f"dec{i}"]
        zs[tag] = {i: v.double().permute(0, 2, 3, 1) for i, v in z.items()}
        if tag == "fp64":
            _, dpred_ref = LM.hourglass_nll(y, pred.numpy(), B, L)
            g64, _ = OE.train_step_grads(P, torch.tensor(x, dtype=dt), torch.tensor(dpred_ref),
                                         drop_scales=drop)
    for i, (conv, bn, skip) in enumerate(eng.dec):
        pre = eng.act[f"dec{i}_pre"].double().cpu()
        # gamma / beta as the forward saw them (the step's Adam update has moved the params)
        ga = torch.tensor(weights[f"dec_bn{i}/gamma"], dtype=torch.float64)
        be = torch.tensor(weights[f"dec_bn{i}/beta"], dtype=torch.float64)
        zh = (pre - bn.mean.double().cpu()) * bn.invstd.double().cpu() * ga + be
        z64 = zs["fp64"][i]
        fl_h = ((zh > 0) != (z64 > 0))
        fl_32 = ((zs["fp32"][i] > 0) != (z64 > 0))
        k = f"dec_bn{i}/beta"
        err = (eng.grads[k].double().cpu() - g64[k]).abs()
        scale = float(g64[k].abs().max())
        worst = int(err.argmax())
        res[f"dec{i}"] = {
            "pixels": int(z64.numel()), "flips_hip": int(fl_h.sum()), "flips_fp32": int(fl_32.sum()),
            "near_zero_1e-5": int((z64.abs() < 1e-5 * float(z64.abs().max())).sum()),
            "beta_err_max_rel": float(err.max()) / scale, "worst_channel": worst,
            "flips_hip_worst_channel": int(fl_h[..., worst].sum()),
            "flips_fp32_worst_channel": int(fl_32[..., worst].sum())}
        print(f"dec{i}", json.dumps(res[f"dec{i}"]), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
