"""The graph-replayed training step equals the eager one, step after step (the bench times the
replay; tests/test_configs_gpu.py checks the eager step against the oracle).

Regression test for the replay drift of round 2: with this ROCm runtime's graph packet capture
(its default) a captured hipMemsetAsync was not ordered before the kernel after it, so the
ListMLE scatter-add landed on a partly cleared gradient buffer (tools/graph_bisect.py isolated
pld_listmle_fwd_bwd; tools/graph_memset_repro.hip reproduces it with the runtime alone). The
library no longer records memset nodes; the test runs with the runtime's default settings."""
import numpy as np
import pytest
import torch

from pldepth_amd.trainer import ReplicaTrainer

pytestmark = pytest.mark.gpu


def _state(t):
    e = t.engine
    d = {"step": t.step_dev.float(), "y": t.y_true, "loss": t.loss, "params": e.params.buf,
         "m": t.m, "v": t.v, "vhat": t.vhat, "stats": e.stats.buf}
    for c in e.convs:
        if c.trainable:
            for k in ("w_nat", "w_dg", "w_nat_x3", "w_dg_x3"):
                if getattr(c, k) is not None:
                    d[f"{c.name}.{k}"] = getattr(c, k)
    for n in e.params.names():
        d["grad." + n] = e.grads[n]
    return {k: v.detach().clone() for k, v in d.items()}


@pytest.mark.parametrize("model", ["ff_effnet", "ff_redweb"])
def test_graph_replay_equals_eager(cuda, model):
    B, H, L, R = 2, 64, 5, 20
    rng = np.random.default_rng(0)
    x = torch.from_numpy(rng.random((B, H, H, 3)).astype(np.float32)).to(cuda)
    gt = torch.from_numpy(rng.random((B, H, H)).astype(np.float32)).to(cuda)
    mask = torch.from_numpy((rng.random((B, H, H)) < 0.9).astype(np.float32)).to(cuda)

    def make():
        t = ReplicaTrainer((H, H, 3), B, L, R, 1, seed=0, model=model)
        t.set_batch(x, gt, mask)
        return t

    a, b = make(), make()
    a.step_eager(0.01)
    b.step_eager(0.01)
    a.capture()
    assert a.graphs is not None
    for i in range(6):
        lr = 0.01 * (1 + i)
        a.step(lr)
        a.synchronize()
        b.step_eager(lr)
        b.synchronize()
        sa, sb = _state(a), _state(b)
        # the ListMLE scatter-add over duplicate pixels uses float atomics: equal up to
        # summation order
        bad = [k for k in sa if not torch.allclose(sa[k], sb[k], rtol=1e-4, atol=1e-6)]
        assert not bad, (i, bad[:10])


def test_redweb_ffl_overlap_equals_single_stream(cuda, fixed_schedules):
    """ff_redweb with the feature-fusion layers' left branches on the FFL side stream (forward
    and backward, RedWebFF.overlap_ffl) takes the same step as with everything on one stream:
    same kernels in the same per-stream order with the same schedules, so only the ListMLE
    scatter-add's atomics may reorder. Eager step, then captured replays."""
    B, H, L, R = 2, 64, 5, 20
    rng = np.random.default_rng(1)
    x = torch.from_numpy(rng.random((B, H, H, 3)).astype(np.float32)).to(cuda)
    gt = torch.from_numpy(rng.random((B, H, H)).astype(np.float32)).to(cuda)
    mask = torch.from_numpy((rng.random((B, H, H)) < 0.9).astype(np.float32)).to(cuda)

    def make(overlap):
        t = ReplicaTrainer((H, H, 3), B, L, R, 1, seed=0, model="ff_redweb")
        t.engine.overlap_ffl = t.engine.overlap_proj = overlap
        t.set_batch(x, gt, mask)
        return t

    a, b = make(1), make(0)
    for t in (a, b):
        t.step_eager(0.01)
        t.synchronize()
    sa, sb = _state(a), _state(b)
    bad = [k for k in sa if not torch.allclose(sa[k], sb[k], rtol=1e-4, atol=1e-6)]
    assert not bad, ("eager", bad[:10])
    a.capture()
    b.capture()
    for i in range(3):
        for t in (a, b):
            t.step(0.01 * (2 + i))
            t.synchronize()
        sa, sb = _state(a), _state(b)
        bad = [k for k in sa if not torch.allclose(sa[k], sb[k], rtol=1e-4, atol=1e-6)]
        assert not bad, (i, bad[:10])
