"""The data-parallel ReplicaTrainer path over the real "nccl" backend (= RCCL) on the one leased
GPU: a single-rank RCCL process group, so RCCL's communicator, its own stream and c10d's stream
dependencies (the side stream's work.wait() on RCCL's stream, then each bucket's Adam) run for
real — with the overlapped exchange (ff_effnet) also the all-reduces issued from the weight-
gradient stream while the encoder backward replays; the multi-rank tests (test_dp_gpu.py) need
gloo because RCCL takes one GPU per rank.

The rank steps through the N > 1 machinery (trainer._step_dp eager, then _capture_dp /
_replay_dp: compute graph, per-bucket all-reduces issued between the update graphs). With one
rank the all-reduce sums one replica, so after 2 steps the parameters must match the plain N = 1
step (trainer._update: one Adam over the whole buffer) of the same batch."""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

B, H, L, R, STEPS = 2, 64, 5, 20, 2


def _data():
    rng = np.random.default_rng(11)
    x = rng.random((B, H, H, 3)).astype(np.float32)
    gt = rng.random((B, H, H)).astype(np.float32)
    mask = (rng.random((B, H, H)) < 0.9).astype(np.float32)
    return x, gt, mask


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(port, q, model, overlap):
    import torch.distributed as dist
    from pldepth_amd import kernels as K
    from pldepth_amd.trainer import ReplicaTrainer
    K.AUTOTUNE = False  # the built-in schedules, as the serial reference uses
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    torch.set_num_threads(1)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        x, gt, mask = _data()
        tr = ReplicaTrainer((H, H, 3), B, L, R, 1, seed=0, rank=0, world_size=1,
                            process_group=dist.group.WORLD, model=model, dp_overlap=overlap)
        assert tr.dp_overlap == overlap
        tr.set_batch(torch.from_numpy(x).cuda(), torch.from_numpy(gt).cuda(),
                     torch.from_numpy(mask).cuda())
        with torch.cuda.stream(tr.stream):
            K.set_scalar(tr.lr_dev, 0.01)
            tr._step_dp()  # eager: backward, bucket all-reduces on RCCL, side-stream Adam
        tr.synchronize()
        g1 = tr.engine.grads.buf.cpu().numpy()
        p1 = tr.engine.params.buf.cpu().numpy()
        tr._capture_dp()  # compute graph + per-bucket update graphs, collectives between them
        assert len(tr.bucket_graphs) >= 2
        for _ in range(STEPS - 1):
            with torch.cuda.stream(tr.stream):
                K.set_scalar(tr.lr_dev, 0.01)
                tr._replay_dp()
        tr.synchronize()
        for w in tr._dp_works:
            w.wait()
        torch.cuda.synchronize()
        q.put((dist.get_backend(), str(torch.cuda.nccl.version()), len(tr.bucket_graphs),
               tr.engine.params.buf.cpu().numpy(), g1, p1, tr.loss_value(),
               int(tr.step_dev.item())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("model,overlap", [("ff_effnet", False), ("ff_effnet", True),
                                           ("ff_redweb", False)])
def test_rccl_single_rank_dp_step_equals_n1_step(cuda, model, overlap):
    """overlap: the decoder buckets' all-reduces issued on RCCL from the weight-gradient stream
    while the encoder backward runs (trainer dp_overlap), as the driver's 8-GPU run does."""
    import torch.multiprocessing as mp
    from pldepth_amd import kernels as K
    from pldepth_amd.trainer import ReplicaTrainer
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rank_main, args=(_free_port(), q, model, overlap))
    p.start()
    backend, version, nbuckets, pb, g1, p1, loss, step = q.get(timeout=240)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert backend == "nccl"
    print(f"RCCL {version}: {nbuckets} buckets")
    # serial reference: the N = 1 step (one Adam over the whole buffer), same schedules
    saved = (K.AUTOTUNE, dict(K._TILE_CACHE))
    K.AUTOTUNE = False
    K._TILE_CACHE.clear()
    try:
        x, gt, mask = _data()
        t = ReplicaTrainer((H, H, 3), B, L, R, 1, seed=0, rank=0, world_size=1, model=model)
        t.set_batch(torch.from_numpy(x).cuda(), torch.from_numpy(gt).cuda(),
                    torch.from_numpy(mask).cuda())
        g_first = p_first = None
        for _ in range(STEPS):
            t.step_eager(0.01)
            t.synchronize()
            if g_first is None:
                g_first = t.engine.grads.buf.cpu().numpy()
                p_first = t.engine.params.buf.cpu().numpy()
    finally:
        K.AUTOTUNE = saved[0]
        K._TILE_CACHE.update(saved[1])
    # as test_dp_gpu.py: ListMLE's float atomics leave rounding noise in gradients that are zero
    # in exact arithmetic, and Adam's first step moves those parameters by ~lr * sign(noise), so
    # step-1 parameters are compared where the gradient is clearly non-zero, step 2 by its loss
    gmax = np.abs(g_first).max()
    solid = np.abs(g_first) > 1e-4 * gmax
    assert solid.mean() > 0.5
    assert step == STEPS + 1
    np.testing.assert_allclose(g1, g_first, rtol=1e-3, atol=1e-4 * gmax)
    np.testing.assert_allclose(p1[solid], p_first[solid], rtol=1e-5, atol=1e-7)
    assert abs(loss - t.loss_value()) <= 1e-3 * abs(loss)
    assert np.isfinite(pb).all()
