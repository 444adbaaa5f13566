"""Experiment: ff_redweb at 448x448 batch 32 — forward error vs fp64 per encoder bf16x3
population threshold, and the eager fwd+bwd time of each."""
import os
import sys
import time

os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")
import numpy as np  # noqa: E402
import torch  # noqa: E402

sys.path.insert(0, ".")
from oracle import redweb as OR  # noqa: E402
from pldepth_amd import kernels as K  # noqa: E402
from pldepth_amd.models.redweb_ff import RedWebFF, preprocess_input  # noqa: E402

torch.cuda.set_device(0)
B, H, R, L = 32, 448, 100, 5
rng = np.random.default_rng(32)
x = preprocess_input(rng.random((B, H, H, 3)).astype(np.float32))
eng = RedWebFF((H, H, 3), B, seed=0, conv_math="auto")
P = {k: torch.tensor(v, dtype=torch.float64) for k, v in eng.get_weights().items()}
taps = {}
t0 = time.time()
with torch.no_grad():
    OR.forward(P, torch.tensor(x, dtype=torch.float64), taps=taps, preprocessed=True)
print("oracle s", time.time() - t0, flush=True)
names = ["conv3_block4_out", "conv4_block3_out", "conv5_block3_out", "ffl0", "ffl1"]
dp = torch.randn(B, H, H, 1, device="cuda") * 1e-3
for thr in [4096, 8192, 16384, 32768, 1 << 40]:
    eng.x3_min_population = thr
    eng.set_weights({k: v.float().numpy() for k, v in P.items()})
    eng.act["input"].copy_(torch.from_numpy(x))
    eng.forward(training=True)
    torch.cuda.synchronize()
    errs = {}
    for n in names:
        mine = eng.act[n if not n.startswith("ffl") else n + "/out"].double().cpu()
        ref = taps[n].permute(0, 2, 3, 1)
        errs[n] = float((mine - ref).abs().max() / ref.abs().max())
    eng.backward(dp)  # tune
    torch.cuda.synchronize()
    t0 = time.time()
    for _ in range(3):
        eng.forward(training=True)
        eng.backward(dp)
    torch.cuda.synchronize()
    print(thr, f"{(time.time() - t0) / 3 * 1e3:.1f} ms", {k: f"{v:.2e}" for k, v in errs.items()},
          flush=True)
