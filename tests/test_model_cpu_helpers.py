"""CPU helpers shared by the data-parallel tests (oracle-only: no GPU)."""
import numpy as np
import torch

from oracle import effnet as OE
from oracle import listmle as LM


def cpu_weights(H=32, seed=0):
    from pldepth_amd.models import effnet_ff as E

    class _CPU(E.EffNetFF):
        def __init__(self):
            self.H, self.W, self.B = H, H, 1
            self.device = torch.device("cpu")
            self.params, self.frozen, self.stats = E.FlatStore(), E.FlatStore(), E.FlatStore()
            self.bns, self.convs = [], []
            self._build_spec()
            for s in (self.params, self.frozen, self.stats):
                s.materialize("cpu")

        def set_weights(self, w):
            for store in (self.params, self.frozen, self.stats):
                for name, shape, _ in store.specs:
                    store[name].copy_(torch.as_tensor(np.asarray(w[name], np.float32)))

    e = _CPU()
    e.init_weights(seed)
    return e.get_weights(), e.params.names()


def shard_grads(rank, world, global_batch=4, H=32, R=6, L=3):
    w, names = cpu_weights(H)
    P = {k: torch.tensor(v, dtype=torch.float64) for k, v in w.items()}
    rng = np.random.default_rng(42)
    x = rng.random((global_batch, H, H, 3))
    idx = rng.integers(0, H * H, (global_batch, R, L))
    lab = -np.sort(-rng.random((global_batch, R, L)), axis=-1)
    y = np.stack([idx, lab], -1).astype(np.float32)
    per = global_batch // world
    sl = slice(rank * per, (rank + 1) * per)
    xs = torch.tensor(x[sl])
    with torch.no_grad():
        pred = OE.forward(P, xs)
    _, dpred = LM.hourglass_nll(y[sl], pred.numpy(), per, L)
    g, _ = OE.train_step_grads(P, xs, torch.tensor(dpred))
    return torch.cat([g[k].flatten() for k in names])
