"""Diagnostic: where along the ff_redweb backward does HIP's gradient leave
the fp64 one, in test_cfg3_redweb_448's case (batch 2, 448x448, 'mixed', built-in schedules)?

For every ReLU site (oracle/redweb.py relu_sites) the HIP gradient w.r.t. the site's output
(engine.gact[site]) is compared with the fp64 oracle's, the oracle run along HIP's own ReLU
branches (flip-aware) and fed HIP's dL/dpred, so that both backward passes start from the same
gradient and take the same branches: what remains is backward arithmetic. Prints the sites in
backward order with their max-relative error; writes gpurun_out/redweb_dz.json.

    python tools/exp_redweb_dz.py
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import redweb as OR  # noqa: E402
from pldepth_amd import kernels as K  # noqa: E402
from pldepth_amd.models.redweb_ff import RedWebFF, preprocess_input  # noqa: E402


def rel(a, b):
    a = torch.as_tensor(a).detach().double().cpu()
    b = torch.as_tensor(b).detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp(min=1e-30))


def main():
    torch.cuda.set_device(0)
    K.AUTOTUNE = False
    K._TILE_CACHE.clear()
    B, H, R, L = 2, 448, 100, 5
    rng = np.random.default_rng(4)
    x = preprocess_input(rng.random((B, H, H, 3)).astype(np.float32))
    math = os.environ.get("PLD_EXP_MATH", "mixed")
    eng = RedWebFF((H, H, 3), B, seed=0, conv_math=math)
    W = eng.get_weights()
    eng.act["input"].copy_(torch.from_numpy(x))
    pred = eng.forward(training=True)
    sites = OR.relu_sites()
    mr = {st: (eng.act[st] > 0).permute(0, 3, 1, 2).cpu() for st in sites}
    # a smooth dL/dpred (no ListMLE): the same for both backward passes
    g = torch.Generator().manual_seed(1)
    dpred = torch.randn(pred.shape, generator=g, dtype=torch.float64) * 1e-3
    eng.backward(dpred.float().cuda())
    torch.cuda.synchronize()
    hip_g = {st: eng.gact[st].permute(0, 3, 1, 2).double().cpu() for st in sites
             if st in eng.gact}
    hip_w = {k: eng.grads[k].detach().double().cpu() for k in OR.trainable_names()}
    # oracle with retained gradients of every ReLU output
    P = {k: torch.tensor(v, dtype=torch.float64) for k, v in W.items()}
    names = set(OR.trainable_names())
    Q = {k: (v.clone().requires_grad_(True) if k in names else v) for k, v in P.items()}
    outs = {}
    bn_in = {}
    orig = OR._relu
    orig_bn = OR._bn

    def bn_keep(P_, name, xx, eps):
        bn_in[name] = xx.detach()
        return orig_bn(P_, name, xx, eps)
    OR._bn = bn_keep

    def relu_keep(xx, site, masks=None, branches=None):
        y = orig(xx, site, masks, branches)
        y.retain_grad()
        outs[site] = y
        return y
    OR._relu = relu_keep
    try:
        out = OR.forward(Q, torch.tensor(x, dtype=torch.float64), preprocessed=True,
                         relu_masks=mr)
        out.backward(dpred)
    finally:
        OR._relu = orig
        OR._bn = orig_bn
    rows = []
    for st in reversed(sites):  # backward order
        if st in hip_g and outs[st].grad is not None:
            rows.append((st, rel(hip_g[st], outs[st].grad)))
    for st, e in rows:
        print(f"{st:40s} {e:.3e}", flush=True)
    werr = {k: rel(hip_w[k], Q[k].grad) for k in names}
    # the fp32 restatements on the SAME problem: HIP's branches, the same dL/dpred
    P32 = {k: torch.tensor(v, dtype=torch.float32) for k, v in W.items()}
    x32 = torch.tensor(x)
    g32 = OR.train_step_grads(P32, x32, dpred.float(), preprocessed=True, relu_masks=mr)[0]
    with torch.backends.mkldnn.flags(enabled=False):
        g32b = OR.train_step_grads(P32, x32, dpred.float(), preprocessed=True, relu_masks=mr)[0]
    e32 = {k: rel(g32[k], Q[k].grad) for k in names}
    e32b = {k: rel(g32b[k], Q[k].grad) for k in names}
    zeros = {"aol/conv0/bias", "aol/conv1/bias", "aol/conv2/bias"}
    keys = [k for k in names if k not in zeros]
    worst = sorted(keys, key=lambda k: -werr[k] / max(e32[k], e32b[k], 1e-12))[:15]
    print("weight gradients, same problem (HIP branches, same dL/dpred): HIP / oneDNN fp32 / "
          "native fp32, worst HIP / worse-fp32 ratio first")
    for k in worst:
        print(f"  {k:40s} {werr[k]:.3e} {e32[k]:.3e} {e32b[k]:.3e}  x{werr[k] / max(e32[k], e32b[k]):.2f}")
    print("tensors over 1e-3: HIP", sum(werr[k] > 1e-3 for k in keys), "oneDNN",
          sum(e32[k] > 1e-3 for k in keys), "native", sum(e32b[k] > 1e-3 for k in keys),
          "of", len(keys))
    # dgamma = sum dz * xhat of the decoder BNs with a ReLU after them, from each side's dz
    # (gradient at the ReLU output x branch mask) and xhat (its own forward): which input
    # carries HIP's error
    print("decoder BN gammas: dgamma from (dz, xhat) of HIP / fp64, error vs fp64's dgamma")
    bns = {}
    for d in eng.ffls:
        for part in ("left", "down"):
            bt = d[part]
            for i, bn in enumerate(bt["bns"]):
                if i % 3 != 2:  # bn0, bn1, bn3, bn4: BN -> ReLU (act site)
                    bns[f"{bt['name']}/bn{i}"] = (bn, f"{bt['name']}/pre{i}", f"{bt['name']}/act{i}")
    for name, (bn, pre, site) in bns.items():
        xh_h = ((eng.act[pre].double() - bn.mean.double()) * bn.invstd.double()).permute(0, 3, 1, 2).cpu()
        xo = bn_in[name]
        mu = xo.mean(dim=(0, 2, 3), keepdim=True)
        var = ((xo - mu) ** 2).mean(dim=(0, 2, 3), keepdim=True)
        xh_o = (xo - mu) / torch.sqrt(var + OR.DEC_BN_EPS)
        m = mr[site].double()
        dz_h = hip_g[site] * m
        dz_o = outs[site].grad * m
        ref = Q[name + "/gamma"].grad
        f = lambda dz, xh: (dz * xh).sum(dim=(0, 2, 3))
        print(f"  {name:28s} HIP {werr[name + '/gamma']:.2e}  (dzH,xhH) {rel(f(dz_h, xh_h), ref):.2e}"
              f"  (dzH,xhO) {rel(f(dz_h, xh_o), ref):.2e}  (dzO,xhH) {rel(f(dz_o, xh_h), ref):.2e}"
              f"  (dzO,xhO) {rel(f(dz_o, xh_o), ref):.2e}  xhat {rel(xh_h, xh_o):.1e} dz {rel(dz_h, dz_o):.1e}",
              flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", f"redweb_dz_{math}.json"), "w") as f:
        json.dump({"sites": rows, "weights": werr, "fp32_onednn": e32, "fp32_native": e32b}, f,
                  indent=1)


if __name__ == "__main__":
    main()
