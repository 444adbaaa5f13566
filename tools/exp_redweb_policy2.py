"""Experiment: ff_redweb at 448x448 batch 32 — forward error vs fp64 per choice of the conv2-stage
convs kept exact fp32 in the forward (RedWebFF.exact_stages; round 3: which of the stage's convs
need it — conv1 / conv2 (3x3) / conv3 / the projection conv0 of each bottleneck), next to the
torch-CPU fp32 restatement's own error on the same input, and the eager fwd+bwd time of each.
Writes gpurun_out/redweb_policy2.json."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from oracle import redweb as OR  # noqa: E402
from pldepth_amd.models.redweb_ff import RedWebFF, preprocess_input  # noqa: E402

torch.cuda.set_device(0)
B, H = 32, 448
rng = np.random.default_rng(32)
x = preprocess_input(rng.random((B, H, H, 3)).astype(np.float32))
eng = RedWebFF((H, H, 3), B, seed=0, conv_math="auto")
W = eng.get_weights()
P = {k: torch.tensor(v, dtype=torch.float64) for k, v in W.items()}
P32 = {k: torch.tensor(v, dtype=torch.float32) for k, v in W.items()}
names = ["conv2_block3_out", "conv3_block4_out", "conv4_block3_out", "conv5_block3_out",
         "ffl0", "ffl1", "ffl2", "pred"]
taps, taps32 = {}, {}
t0 = time.time()
with torch.no_grad():
    taps["pred"] = OR.forward(P, torch.tensor(x, dtype=torch.float64), taps=taps,
                              preprocessed=True)
    print("oracle fp64 s", time.time() - t0, flush=True)
    taps32["pred"] = OR.forward(P32, torch.tensor(x), taps=taps32, preprocessed=True)
print("oracle fp32 s", time.time() - t0, flush=True)


def ref_nhwc(t, n):
    return t if n == "pred" else t.permute(0, 2, 3, 1)


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).abs().max() / b.abs().max())


out = {"fp32_restatement": {n: rel(ref_nhwc(taps32[n], n), ref_nhwc(taps[n], n))
                            for n in names}}
print("fp32", {k: f"{v:.2e}" for k, v in out["fp32_restatement"].items()}, flush=True)
del taps32


def mine(n):
    if n == "pred":
        return eng.act["pred"]
    return eng.act[n if not n.startswith("ffl") else n + "/out"]


dp = torch.randn(B, H, H, 1, device="cuda") * 1e-3
def blk(*sufs):
    return tuple(f"conv2_block{i}_{x}" for i in (1, 2, 3) for x in sufs)


VARIANTS = [("conv2", ("conv2",)), ("c2", blk("2")), ("c1c2", blk("1", "2")),
            ("c2c3", blk("2", "3")), ("c2c3c0", blk("2", "3", "0")), ("none", ())]
for thr, stages in VARIANTS:
    eng.exact_stages = stages
    eng.set_weights(W)
    eng.act["input"].copy_(torch.from_numpy(x))
    eng.forward(training=True)
    torch.cuda.synchronize()
    errs = {n: rel(mine(n), ref_nhwc(taps[n], n)) for n in names}
    eng.backward(dp)  # tune
    torch.cuda.synchronize()
    t0 = time.time()
    for _ in range(3):
        eng.forward(training=True)
        eng.backward(dp)
    torch.cuda.synchronize()
    ms = (time.time() - t0) / 3 * 1e3
    out[str(thr)] = {"ms": ms, "errors": errs}
    print(thr, f"{ms:.1f} ms", {k: f"{v:.2e}" for k, v in errs.items()}, flush=True)
os.makedirs("gpurun_out", exist_ok=True)
with open("gpurun_out/redweb_policy2.json", "w") as f:
    json.dump(out, f, indent=1)
