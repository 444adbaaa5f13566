"""Multi-process data-parallel tests on CPU (gloo, world_size 2): the gradient exchange and the
replica semantics the GPU path uses (per-replica BN statistics, mean of replica gradients)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from pldepth_amd import dp
from pldepth_amd.dp import allreduce_bucket, shard, tensor_buckets


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


def _exchange(flat, offsets, bucket_bytes, group=None):
    """The trainer's exchange (trainer._dp_exchange): every tensor-aligned bucket all-reduced
    async in reverse order, then waited on."""
    buckets = tensor_buckets(offsets, flat.numel(), bucket_bytes)
    works = [allreduce_bucket(flat, lo, hi, group) for lo, hi in buckets]
    for w in works:
        w.wait()
    return buckets


def _bucketed_sum(rank, world):
    g = torch.arange(1003, dtype=torch.float32) * (rank + 1)
    buckets = _exchange(g, [990, 900, 700, 640, 300, 100, 5], bucket_bytes=256)
    return g.numpy(), buckets


def test_bucketed_allreduce_sums_every_element():
    out = _spawn(_bucketed_sum)
    ref = np.arange(1003, dtype=np.float32) * 3
    for r in (0, 1):
        np.testing.assert_array_equal(out[r][0], ref)
    # >= 64 floats per bucket, boundaries at tensor starts; offset 0 closes the last one
    assert out[0][1] == [(900, 1003), (700, 900), (300, 700), (100, 300), (5, 100), (0, 5)]
    assert out[0][1] == out[1][1]


def test_tensor_buckets_tile_the_buffer():
    rng = np.random.default_rng(3)
    for _ in range(50):
        n = int(rng.integers(1, 10000))
        offs = sorted(set(rng.integers(0, n, int(rng.integers(0, 40))).tolist()))
        got = tensor_buckets(offs, n, bucket_bytes=int(rng.integers(4, 4000)))
        assert got[0][1] == n and got[-1][0] == 0
        assert all(a[0] == b[1] for a, b in zip(got, got[1:]))  # contiguous, reverse order
        assert all(lo < hi for lo, hi in got)
        starts = set(offs) | {0}
        assert all(lo in starts for lo, _ in got)  # no tensor spans two buckets
    with pytest.raises(ValueError):
        tensor_buckets([10], 10)


def test_shard_layout():
    assert shard(256, 0, 8) == (0, 32) and shard(256, 7, 8) == (224, 32)
    with pytest.raises(ValueError):
        shard(10, 0, 4)


def _replica_grads(rank, world):
    """Each replica: oracle fp64 gradient of ITS shard's mean ListMLE loss (BN statistics over
    its own images), then the all-reduced mean — what every GPU applies in Adam."""
    from tests.test_model_cpu_helpers import shard_grads
    flat = shard_grads(rank, world)
    _exchange(flat, [], bucket_bytes=64 << 20)
    flat /= world
    return flat[::97].numpy().copy(), float(flat.sum())  # keep the IPC message small


def test_replica_gradients_average_matches_serial_shards():
    out = _spawn(_replica_grads)
    from tests.test_model_cpu_helpers import shard_grads
    serial = (shard_grads(0, 2) + shard_grads(1, 2)) / 2
    np.testing.assert_allclose(out[0][0], serial[::97].numpy(), rtol=1e-12, atol=1e-15)
    assert abs(out[0][1] - float(serial.sum())) <= 1e-9 * float(serial.abs().sum())
    np.testing.assert_array_equal(out[0][0], out[1][0])  # replicas stay bit-identical


def _checksums(rank, world):
    same = torch.linspace(-3, 3, 5000)
    ok_same, sums = dp.replicas_identical(same)
    other = same.clone()
    if rank == 1:
        other[4321] = torch.nextafter(other[4321], torch.tensor(10.0))  # one ulp on one rank
    ok_other, _ = dp.replicas_identical(other)
    swapped = same.clone()
    if rank == 1:  # same values, two of them exchanged: the position weights catch it
        swapped[[10, 20]] = swapped[[20, 10]]
    ok_swapped, _ = dp.replicas_identical(swapped)
    return ok_same, ok_other, ok_swapped, sums


def test_replicas_identical_gloo():
    out = _spawn(_checksums)
    for r in (0, 1):
        assert out[r][:3] == (True, False, False)
        assert out[r][3]["min"] == out[r][3]["max"]


def _dead_rank_job(rank, world, port, q):
    """bench.py's multi-rank structure on gloo: bounded init, the run inside exit_on_failure,
    rank 1 dying after the rendezvous, rank 0 then entering its first collective."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank))
    torch.set_num_threads(1)
    import time

    def run():
        dp.init_group("gloo", rank, world, timeout_s=20)
        if rank == 1:
            os._exit(3)
        time.sleep(1.0)
        dp.replicas_identical(torch.ones(100))  # the peer is gone: raises
        q.put("unreachable")
    dp.exit_on_failure(run, world)


def test_dead_rank_makes_survivor_exit_nonzero():
    import time
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    t0 = time.time()
    ps = [ctx.Process(target=_dead_rank_job, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(timeout=120)
    alive = [p.is_alive() for p in ps]
    for p in ps:
        if p.is_alive():
            p.kill()
    assert not any(alive), "a rank is still blocked after the timeout"
    assert ps[1].exitcode == 3
    assert ps[0].exitcode not in (0, None)
    assert time.time() - t0 < 100
    assert q.empty()


def test_rccl_version_is_string_or_none():
    v = dp.rccl_version()
    assert v is None or (isinstance(v, str) and v.count(".") >= 1)
