"""Debug: which part of the step differs between hipGraph replay and eager execution."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from pldepth_amd import kernels as K
from pldepth_amd.models.effnet_ff import EffNetFF

torch.cuda.set_device(0)
B, H, L, R = 2, 64, 5, 20
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


def fwd():
    eng.forward(training=True, step=1)


def lossf():
    K.listmle_fwd_bwd(eng.act["pred"], y, B, R, L, dpred=dpred, nll=nll, loss=loss,
                      zero_dpred=True)


def bwd():
    eng.backward(dpred)


def snap():
    torch.cuda.synchronize()
    return {"pred": eng.act["pred"].clone(), "loss": loss.clone(), "dpred": dpred.clone(),
            "grads": eng.grads.buf.clone(), "g_top": eng.gact["top_activation"].clone(),
            "g_dec4": eng.gact["dec4_up"].clone()}


def compare(tag, a, b):
    out = []
    for k in a:
        d = float((a[k] - b[k]).abs().max())
        s = float(b[k].abs().max())
        out.append(f"{k}={d:.3g}/{s:.3g}")
    print(tag, " ".join(out), flush=True)


with torch.cuda.stream(st):
    fwd(); lossf(); bwd()
ref = snap()
for name, fn in [("bwd", bwd), ("loss+bwd", lambda: (lossf(), bwd())),
                 ("fwd+loss+bwd", lambda: (fwd(), lossf(), bwd()))]:
    with torch.cuda.stream(st):
        fwd(); lossf()
        eng.grads.buf.fill_(float("nan"))
        for t in eng.gact.values():
            t.fill_(float("nan"))
        if name == "fwd+loss+bwd":
            eng.act["pred"].fill_(float("nan"))
        torch.cuda.synchronize()
        g = K.Graph().capture(fn)
        torch.cuda.synchronize()
        g.launch()
    compare(name, snap(), ref)
    del g

bad = [n for n in eng.params.names() if not torch.isfinite(eng.grads[n]).all()]
print("NaN grads after last replay:", len(bad), bad[:40])
