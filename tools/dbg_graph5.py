"""Debug: graph replay vs eager, strictly sequential (synchronize between trainers), with and
without allocations between capture and replay."""
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


def make():
    t = ReplicaTrainer((H, H, 3), B, L, R, 1, seed=0)
    t.set_batch(x, gt, mask)
    torch.cuda.synchronize()
    return t


def snap(t):
    torch.cuda.synchronize()
    e = t.engine
    return {"loss": t.loss.clone(),
            "grads": torch.cat([e.grads[n].flatten() for n in e.params.names()]),
            "params": torch.cat([e.params[n].flatten() for n in e.params.names()])}


def cmp(tag, a, b):
    print(tag, " ".join(f"{k}={float((a[k] - b[k]).abs().max()):.3g}/"
                        f"{float(b[k].abs().max()):.3g}" for k in a), flush=True)


A, Bt = make(), make()
A.step_eager(0.01); torch.cuda.synchronize()
Bt.step_eager(0.01); torch.cuda.synchronize()
cmp("step1 eager/eager", snap(A), snap(Bt))
A.capture()
for i in range(2, 5):
    A.step(0.01); A.synchronize(); torch.cuda.synchronize()
    Bt.step_eager(0.01); Bt.synchronize(); torch.cuda.synchronize()
    cmp(f"step{i} graph/eager", snap(A), snap(Bt))
    ea, eb = A.engine, Bt.engine
    bad = [n for n in ea.params.names()
           if float((ea.grads[n] - eb.grads[n]).abs().max()) > 1e-3 * float(eb.grads[n].abs().max()) + 1e-12]
    print("  bad grads:", len(bad), bad[:12])
    badg = [k for k in ea.gact if float((ea.gact[k] - eb.gact[k]).abs().max()) >
            1e-3 * float(eb.gact[k].abs().max()) + 1e-12]
    print("  bad gact:", len(badg), badg[:12])
    bada = [k for k in ea.act if float((ea.act[k] - eb.act[k]).abs().max()) >
            1e-3 * float(eb.act[k].abs().max()) + 1e-12]
    print("  bad act:", len(bada), bada[:12])
    badp = [k for k, v in ea._gpre.items() if float((v - eb._gpre[k]).abs().max()) >
            1e-3 * float(eb._gpre[k].abs().max()) + 1e-12]
    print("  bad gpre:", badp)
junk = [torch.full((n,), float("nan"), device="cuda") for n in
        [64, 256, 1024, 4096, 1 << 14, 1 << 16, 1 << 18, 1 << 20, 1 << 22] for _ in range(8)]
torch.cuda.synchronize()
for i in range(5, 7):
    A.step(0.01); A.synchronize(); torch.cuda.synchronize()
    Bt.step_eager(0.01); Bt.synchronize(); torch.cuda.synchronize()
    cmp(f"step{i} graph/eager after junk", snap(A), snap(Bt))
