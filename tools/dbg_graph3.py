"""Debug: trainer phases under hipGraph replay vs eager, phase by phase."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from pldepth_amd import kernels as K
from pldepth_amd.trainer import ReplicaTrainer

torch.cuda.set_device(0)
B, H, L, R = 2, 64, 5, 20
rng = np.random.default_rng(0)
x = torch.from_numpy(rng.random((B, H, H, 3)).astype(np.float32)).cuda()
gt = torch.from_numpy(rng.random((B, H, H)).astype(np.float32)).cuda()
mask = torch.ones(B, H, H).cuda()


def make():
    t = ReplicaTrainer((H, H, 3), B, L, R, 1, seed=0)
    t.set_batch(x, gt, mask)
    torch.cuda.synchronize()
    return t


def snap(t):
    torch.cuda.synchronize()
    e = t.engine
    return {"y": t.y_true.clone(), "pred": e.act["pred"].clone(), "loss": t.loss.clone(),
            "grads": torch.cat([e.grads[n].flatten() for n in e.params.names()]),
            "params": torch.cat([e.params[n].flatten() for n in e.params.names()]),
            "step": t.step_dev.clone().float()}


def cmp(tag, a, b):
    print(tag, " ".join(f"{k}={float((a[k] - b[k]).abs().max()):.3g}/"
                        f"{float(b[k].abs().max()):.3g}" for k in a), flush=True)


phases = {"sample": lambda t: t._sample(), "fwd_bwd": lambda t: t._fwd_bwd(),
          "update": lambda t: t._update()}
for split in (["sample", "fwd_bwd", "update"], ["all"]):
    A, Bt = make(), make()
    A.step_eager(0.01)
    Bt.step_eager(0.01)
    cmp("after eager step 1 (A vs B)", snap(A), snap(Bt))
    for ph in split:
        fns = list(phases.values()) if ph == "all" else [phases[ph]]
        with torch.cuda.stream(A.stream):
            K.set_scalar(A.lr_dev, 0.01)
            torch.cuda.synchronize()
            g = K.Graph().capture(lambda: [f(A) for f in fns])
            torch.cuda.synchronize()
            g.launch()
        with torch.cuda.stream(Bt.stream):
            K.set_scalar(Bt.lr_dev, 0.01)
            for f in fns:
                f(Bt)
        cmp(f"phase {ph}: graph(A) vs eager(B)", snap(A), snap(Bt))
        del g
