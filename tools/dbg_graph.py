"""Debug: graph replay vs eager step, with junk allocations between capture and replay."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from pldepth_amd.trainer import ReplicaTrainer

torch.cuda.set_device(0)
B, H, L, R = 2, 64, 5, 20
mode = sys.argv[1] if len(sys.argv) > 1 else "junk"
rng = np.random.default_rng(0)
x = torch.from_numpy(rng.random((B, H, H, 3)).astype(np.float32)).cuda()
gt = torch.from_numpy(rng.random((B, H, H)).astype(np.float32)).cuda()
mask = torch.ones(B, H, H).cuda()
A = ReplicaTrainer((H, H, 3), B, L, R, 1, seed=0)
A.set_batch(x, gt, mask)
A.step_eager(0.01)
A.capture()
Bt = ReplicaTrainer((H, H, 3), B, L, R, 1, seed=0)
Bt.set_batch(x, gt, mask)
Bt.step_eager(0.01)
junk = []
if mode == "junk":
    for sz in [64, 256, 1024, 4096, 1 << 14, 1 << 16, 1 << 18, 1 << 20, 1 << 22]:
        for _ in range(8):
            junk.append(torch.full((sz,), float("nan"), device="cuda"))
torch.cuda.synchronize()
A.step(0.01)
Bt.step_eager(0.01)
torch.cuda.synchronize()
print("loss", A.loss_value(), Bt.loss_value())
ga, gb = A.engine.grads, Bt.engine.grads
bad = []
for name in A.engine.params.names():
    a, b = ga[name], gb[name]
    e = float((a - b).abs().max() / b.abs().max().clamp(min=1e-30))
    if not (e < 1e-3):
        bad.append((name, e))
print("bad grads:", len(bad), "of", len(A.engine.params.names()))
for n, e in bad[:15]:
    print("  ", n, e)
print("pred diff", float((A.engine.act["pred"] - Bt.engine.act["pred"]).abs().max()))
for k in ["dec4_up", "dec0_up", "top_activation", "block6a_expand_activation"]:
    print("gact", k, float((A.engine.gact[k] - Bt.engine.gact[k]).abs().max()),
          float(Bt.engine.gact[k].abs().max()))
