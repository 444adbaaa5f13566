"""Which conv arithmetic sets the batch-32 ff_effnet decoder gradients' distance from fp64?

The bench step (448x448, batch 32, drop-connect off) is run on the GPU under several conv
arithmetic assignments on identical inputs / weights / rankings, and every trainable gradient
is compared with the fp64 oracle (oracle/effnet.py + oracle/listmle.py, computed once). Prints
the listed tensors' errors and the global rel-L2 per variant (tools/diag_dec_wgrad.py showed
the dW kernels' own arithmetic at ~1e-6: the error is in their operands).

    python tools/exp_dec_precision.py [--schedules PATH] [--out FILE]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

WATCH = ["dec_conv4/kernel", "dec_conv3/kernel", "dec_bn3/gamma", "dec_bn4/beta",
         "dec_conv2/kernel", "dec_conv0/kernel"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--schedules", default="")
    ap.add_argument("--out", default="")
    ap.add_argument("--variants", 
                    default="auto,auto2,dec_fp32,dec01_fp32,dec01_fwd,dec01_bwd,dec0_fwd,dec1_fwd,"
                            "dec2_fwd,mixed")
    a = ap.parse_args()
    from oracle import effnet as OE
    from pldepth_amd import kernels as K
    from pldepth_amd.models.effnet_ff import EffNetFF
    from tests.test_configs_gpu import _oracle_step, make_rankings
    if a.schedules:
        print("schedule entries:", K.use_schedule_table(a.schedules), flush=True)
    torch.cuda.set_device(0)
    B, H, R, L = 32, 448, 100, 5
    rng = np.random.default_rng(32)
    x = rng.random((B, H, H, 3)).astype(np.float32)
    y = make_rankings(rng, B, H, H, R, L)
    res, weights = {}, None
    print("variants: auto = the bench policy; autoN = a repeat (run-to-run spread)", flush=True)
    for var in a.variants.split(","):
        policy = {"mixed": "mixed", "fp32": "fp32"}.get(var.rstrip("0123456789"), "auto")
        eng = EffNetFF((H, H, 3), B, seed=0, conv_math=policy)
        eng.drop_connect = False
        print(var, "enc", eng.enc_math, "dec", eng.dec_math, flush=True)
        if var == "dec_fp32":
            eng.dec_math = "fp32"
        if var.startswith("dec") and var != "dec_fp32":
            # decNN_fp32: decoder convs N.. fp32 forward + backward; decNN_fwd / decNN_bwd: one
            # direction only
            idx = {int(c): "fp32" for c in var[3:var.index("_")]}
            if not var.endswith("_bwd"):
                eng.dec_math_fwd = dict(idx)
            if not var.endswith("_fwd"):
                eng.dec_math_bwd = dict(idx)
        weights = eng.get_weights()
        eng.act["input"].copy_(torch.from_numpy(x))
        pred = eng.forward(training=True)
        _, dpred, _ = K.listmle_fwd_bwd(pred, torch.from_numpy(y).cuda(), B, R, L)
        eng.backward(dpred)
        torch.cuda.synchronize()
        res[var] = {k: eng.grads[k].detach().cpu().double() for k in OE.trainable_names(weights)}
        if var == "auto":  # the BN statistics of the decoder stages (batch mean / invstd)
            bnstat = {i: (bn.mean.double().cpu(), bn.invstd.double().cpu())
                      for i, (_, bn, _) in enumerate(eng.dec)}
        del eng, pred, dpred
        torch.cuda.empty_cache()
        print("ran", var, flush=True)
    torch.set_num_threads(16)
    P = {k: torch.tensor(v, dtype=torch.float64) for k, v in weights.items()}
    _, _, _, g64 = _oracle_step(OE, P, torch.tensor(x, dtype=torch.float64), y, B, L)
    print("oracle done", flush=True)
    keys = [k for k in g64 if not (k.startswith("dec_conv") and k.endswith("/bias"))
            and not k.endswith("project_bn/beta")]
    ref = torch.cat([g64[k].double().flatten() for k in keys])
    out = {}
    for var, g in res.items():
        e = {k: float((g[k] - g64[k]).abs().max() / g64[k].abs().max()) for k in keys}
        flat = torch.cat([g[k].flatten() for k in keys])
        glob = float((flat - ref).norm() / ref.norm())
        out[var] = {"global_rel_l2": glob, "watch": {k: e[k] for k in WATCH},
                    "within_1e-3": sum(v <= 1e-3 for v in e.values())}
        print(var, json.dumps(out[var]), flush=True)
    # per output channel of dec_conv4/kernel: where the auto run's error sits, against the
    # channel's BN-4 statistics (mean / std of dec4_pre) and its gradient magnitude
    if "auto" in res:
        k = "dec_conv4/kernel"
        ref, hip = g64[k].double(), res["auto"][k]
        mx = float(ref.abs().max())
        per = ((hip - ref).abs().amax(dim=(0, 1, 2)) / mx).tolist()
        mag = (ref.abs().amax(dim=(0, 1, 2)) / mx).tolist()
        mean, invstd = bnstat[4]
        print("cout  err/max|ref|  max|ref_c|/max|ref|  bn4 |mean|/std")
        for c in sorted(range(len(per)), key=lambda c: -per[c])[:8]:
            print(f"{c:4d}  {per[c]:.3e}  {mag[c]:.3e}  {abs(float(mean[c])) * float(invstd[c]):.2f}")
        for i in range(4):
            m, s_ = bnstat[i]
            r = (m.abs() * s_)
            print(f"bn{i}: |mean|/std max {float(r.max()):.2f} median {float(r.median()):.2f}")
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
