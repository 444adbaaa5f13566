"""Debug: full trainer step graph vs eager over several steps; report the first differing state."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from pldepth_amd.trainer import ReplicaTrainer

torch.cuda.set_device(0)
B, H, L, R = 2, 64, 5, 20
rng = np.random.default_rng(0)
x = torch.from_numpy(rng.random((B, H, H, 3)).astype(np.float32)).cuda()
gt = torch.from_numpy(rng.random((B, H, H)).astype(np.float32)).cuda()
mask = torch.ones(B, H, H).cuda()
drop = sys.argv[1] != "nodrop" if len(sys.argv) > 1 else True


def make():
    t = ReplicaTrainer((H, H, 3), B, L, R, 1, seed=0, drop_connect=drop)
    t.set_batch(x, gt, mask)
    torch.cuda.synchronize()
    return t


def state(t):
    e = t.engine
    d = {"step": t.step_dev.float(), "draws": t.draws.float(), "y": t.y_true,
         "dpred": t.dpred, "loss": t.loss, "params": e.params.buf, "m": t.m, "v": t.v}
    for c in e.convs:
        if c.trainable:
            for k in ("w_nat", "w_dg", "w_nat_x3", "w_dg_x3"):
                if getattr(c, k) is not None:
                    d[f"{c.name}.{k}"] = getattr(c, k)
    for bi, blk in enumerate(e.blocks):
        d[f"drop{bi}"] = blk["drop"]
    for k, v in e.act.items():
        d["act." + k] = v
    for k, v in e.gact.items():
        d["gact." + k] = v
    d["grads"] = e.grads.buf
    return {k: v.detach().clone() for k, v in d.items()}


A, Bt = make(), make()
A.step_eager(0.01)
A.synchronize()
Bt.step_eager(0.01)
Bt.synchronize()
A.capture()
for i in range(2, 8):
    sa0, sb0 = state(A), state(Bt)
    A.step(0.01)
    A.synchronize()
    torch.cuda.synchronize()
    Bt.step_eager(0.01)
    Bt.synchronize()
    torch.cuda.synchronize()
    sa, sb = state(A), state(Bt)
    bad = [k for k in sa if float((sa[k] - sb[k]).abs().max()) > 1e-4 * float(sb[k].abs().max()) + 1e-12
           or not torch.isfinite(sa[k]).all()]
    print(f"step {i}: {len(bad)} differing: {bad[:25]}", flush=True)
    if bad:
        break
