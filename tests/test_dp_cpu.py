"""Multi-process data-parallel tests on CPU (gloo, world_size 2): the gradient exchange and the
replica semantics the GPU path uses (per-replica BN statistics, mean of replica gradients)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from pldepth_amd.dp import GradientAllReducer, shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(rank, world, port, fn, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)  # OpenMP intra-op pools deadlock in spawned gloo workers here
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank, fn(rank, world)))
    finally:
        dist.destroy_process_group()


def _spawn(fn, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_run, args=(r, world, port, fn, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = dict(q.get(timeout=300) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


def _bucketed_sum(rank, world):
    g = torch.arange(1003, dtype=torch.float32) * (rank + 1)
    GradientAllReducer(g, bucket_bytes=256)()  # 4 buckets of 64 floats... ragged tail
    return g.numpy()


def test_bucketed_allreduce_sums_every_element():
    out = _spawn(_bucketed_sum)
    ref = np.arange(1003, dtype=np.float32) * 3
    for r in (0, 1):
        np.testing.assert_array_equal(out[r], ref)


def test_shard_layout():
    assert shard(256, 0, 8) == (0, 32) and shard(256, 7, 8) == (224, 32)
    with pytest.raises(ValueError):
        shard(10, 0, 4)


def _replica_grads(rank, world):
    """Each replica: oracle fp64 gradient of ITS shard's mean ListMLE loss (BN statistics over
    its own images), then the all-reduced mean — what every GPU applies in Adam."""
    from tests.test_model_cpu_helpers import shard_grads
    flat = shard_grads(rank, world)
    GradientAllReducer(flat)()
    flat /= world
    return flat[::97].numpy().copy(), float(flat.sum())  # keep the IPC message small


def test_replica_gradients_average_matches_serial_shards():
    out = _spawn(_replica_grads)
    from tests.test_model_cpu_helpers import shard_grads
    serial = (shard_grads(0, 2) + shard_grads(1, 2)) / 2
    np.testing.assert_allclose(out[0][0], serial[::97].numpy(), rtol=1e-12, atol=1e-15)
    assert abs(out[0][1] - float(serial.sum())) <= 1e-9 * float(serial.abs().sum())
    np.testing.assert_array_equal(out[0][0], out[1][0])  # replicas stay bit-identical
