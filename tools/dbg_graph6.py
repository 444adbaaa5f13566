"""Debug: replay one captured graph many times on identical inputs; every replay must equal the
eager reference (a race inside the replayed graph shows up as a differing replay)."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from pldepth_amd import kernels as K
from pldepth_amd.models.effnet_ff import EffNetFF

torch.cuda.set_device(0)
B, H, L, R = 2, int(sys.argv[2]) if len(sys.argv) > 2 else 64, 5, 20
rng = np.random.default_rng(0)
eng = EffNetFF((H, H, 3), B, seed=0)
eng.drop_connect = False
eng.act["input"].copy_(torch.from_numpy(rng.random((B, H, H, 3)).astype(np.float32)))
idx = rng.integers(0, H * H, (B, R, L)).astype(np.float32)
lab = -np.sort(-rng.random((B, R, L)), -1).astype(np.float32)
y = torch.from_numpy(np.stack([idx, lab], -1)).cuda()
st = torch.cuda.Stream()
dpred = torch.empty(B, H, H, 1, device="cuda")
nll = torch.empty(B * R, device="cuda")
loss = torch.zeros(1, device="cuda")
names = eng.params.names()


def fwd():
    eng.forward(training=True, step=1)


def lossf():
    K.listmle_fwd_bwd(eng.act["pred"], y, B, R, L, dpred=dpred, nll=nll, loss=loss,
                      zero_dpred=True)


def bwd():
    eng.backward(dpred)


def grads():
    torch.cuda.synchronize()
    return torch.cat([eng.grads[n].flatten() for n in names]).clone()


variants = {"bwd": bwd, "loss+bwd": lambda: (lossf(), bwd()),
            "fwd+loss+bwd": lambda: (fwd(), lossf(), bwd()),
            "fwd": fwd, "dec_bwd_only": None}
which = sys.argv[1] if len(sys.argv) > 1 else "all"
with torch.cuda.stream(st):
    fwd(); lossf(); bwd()
ref = grads()
with torch.cuda.stream(st):
    fwd(); lossf(); bwd()
print("eager repeat diff", float((grads() - ref).abs().max()), "scale", float(ref.abs().max()))
for name, fn in variants.items():
    if fn is None or (which != "all" and which != name):
        continue
    with torch.cuda.stream(st):
        fwd(); lossf()
        torch.cuda.synchronize()
        g = K.Graph().capture(fn)
        torch.cuda.synchronize()
        diffs = []
        for r in range(12):
            g.launch()
            if name == "fwd":
                bwd()
            diffs.append(float((grads() - ref).abs().max()))
    print(name, "replay diffs:", " ".join(f"{d:.2g}" for d in diffs), flush=True)
    del g
