"""Data-parallel plumbing: one process per GPU, torch.distributed ("nccl" = RCCL over xGMI on
ROCm, "gloo" on CPU for tests).

The reference trains on one device; the build shards HR-WSI-shaped minibatches:
rank r owns images [r*B, (r+1)*B) of the global batch (contiguous), draws its rankings and
drop-connect masks from Philox counters keyed by the GLOBAL image index (so results do not
depend on the GPU count), keeps BN statistics per replica (TF MirroredStrategy semantics) and
exchanges exactly one thing per step: the fp32 gradient, summed by all-reduce (buckets of
``bucket_bytes``) and averaged inside the Adam kernel (grad_scale = 1/world).
"""
import os

import torch


def env_rank_world():
    return int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")), \
        int(os.environ.get("LOCAL_RANK", "0"))


def shard(global_batch, rank, world):
    """(first global image, images on this rank) for an evenly divisible global batch."""
    if global_batch % world:
        raise ValueError(f"global batch {global_batch} not divisible by {world} ranks")
    per = global_batch // world
    return rank * per, per


class GradientAllReducer(object):
    """Sum-all-reduce of a flat gradient buffer in fixed-size buckets (async, then wait).

    On RCCL the buckets pipeline over the xGMI links; with one bucket the call is a single
    ncclAllReduce. Works on any backend (gloo for CPU tests)."""

    def __init__(self, flat, group=None, bucket_bytes=64 << 20):
        self.flat = flat
        self.group = group
        n = flat.numel()
        per = max(1, bucket_bytes // flat.element_size())
        self.buckets = [flat[i:i + per] for i in range(0, n, per)]

    def __call__(self):
        import torch.distributed as dist
        handles = [dist.all_reduce(b, group=self.group, async_op=True) for b in self.buckets]
        for h in handles:
            h.wait()
        return self.flat


def average_(flat, world):
    """In-place mean for backends/tests that reduce outside the Adam kernel."""
    if world > 1:
        flat.div_(world)
    return flat


def is_distributed():
    try:
        import torch.distributed as dist
        return dist.is_available() and dist.is_initialized()
    except Exception:
        return False


__all__ = ["env_rank_world", "shard", "GradientAllReducer", "average_", "is_distributed",
           "torch"]
