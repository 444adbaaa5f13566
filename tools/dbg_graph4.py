"""Debug: allocations made during hipGraph capture (dangling once freed)."""
import sys
import traceback

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
A = ReplicaTrainer((H, H, 3), B, L, R, 1, seed=0)
A.set_batch(x, gt, mask)
A.step_eager(0.01)
torch.cuda.synchronize()

# trace every torch allocation made while capturing
orig_empty, orig_empty_like, orig_zeros = torch.empty, torch.empty_like, torch.zeros
log = []


def wrap(fn, name):
    def w(*a, **k):
        t = fn(*a, **k)
        if getattr(t, "is_cuda", False):
            log.append((name, tuple(t.shape), "".join(traceback.format_stack(limit=6)[:-1])))
        return t
    return w


s0 = torch.cuda.memory_stats()["allocation.all.allocated"]
torch.empty, torch.empty_like, torch.zeros = (wrap(orig_empty, "empty"),
                                              wrap(orig_empty_like, "empty_like"),
                                              wrap(orig_zeros, "zeros"))
try:
    A.capture()
finally:
    torch.empty, torch.empty_like, torch.zeros = orig_empty, orig_empty_like, orig_zeros
s1 = torch.cuda.memory_stats()["allocation.all.allocated"]
print("allocations during capture:", s1 - s0, "traced:", len(log))
for name, shape, stack in log[:10]:
    print(name, shape)
    print(stack)
