"""Data-parallel plumbing: one process per GPU, torch.distributed ("nccl" = RCCL over xGMI on
ROCm, "gloo" on CPU for tests).

The reference trains on one device; the build shards HR-WSI-shaped minibatches:
rank r owns images [r*B, (r+1)*B) of the global batch (contiguous), draws its rankings and
drop-connect masks from Philox counters keyed by the GLOBAL image index (so results do not
depend on the GPU count), keeps BN statistics per replica (TF MirroredStrategy semantics) and
exchanges exactly one thing per step: the fp32 gradient, summed by all-reduce in reverse-order,
tensor-aligned buckets (``tensor_buckets``) and averaged inside the Adam kernel (grad_scale =
1/world). ``ReplicaTrainer`` (trainer.py) issues them after its (graph-replayed) backward, each
bucket's Adam-AMSGrad + filter refresh running on a side stream as soon as that bucket lands,
i.e. the exchange overlaps the optimizer step.
"""
import os


def env_rank_world():
    return int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")), \
        int(os.environ.get("LOCAL_RANK", "0"))


def shard(global_batch, rank, world):
    """(first global image, images on this rank) for an evenly divisible global batch."""
    if global_batch % world:
        raise ValueError(f"global batch {global_batch} not divisible by {world} ranks")
    per = global_batch // world
    return rank * per, per


def tensor_buckets(offsets, numel, bucket_bytes=8 << 20, elem_bytes=4):
    """Reverse-order buckets of a flat gradient buffer, aligned to tensor starts.

    offsets: flat start offsets of the parameter tensors (any order). Tensors are grouped from
    the end of the buffer towards offset 0 (the order the backward finalises them) into buckets
    of at least `bucket_bytes` (the last one, at offset 0, may be smaller; a tensor larger than
    a bucket is a bucket of its own). No tensor spans two buckets, so a bucket's optimizer
    update can refresh the derived copies (native conv filters) of every tensor in it. The
    buckets tile [0, numel) exactly. ~8 MB: large enough that each RCCL ring all-reduce runs at
    link rate over xGMI (7 x ~153 GB/s point-to-point links), small enough that the updates of
    the first buckets overlap the all-reduces of the later ones."""
    starts = sorted(set(int(o) for o in offsets) | {0})
    if starts[-1] >= numel:
        raise ValueError("tensor offset beyond the buffer")
    buckets, hi = [], int(numel)
    for lo in reversed(starts):
        if (hi - lo) * elem_bytes >= bucket_bytes or lo == 0:
            buckets.append((lo, hi))
            hi = lo
    return buckets


def allreduce_bucket(flat, lo, hi, group=None):
    """Async sum-all-reduce of flat[lo:hi] (ordered after the caller's current stream by
    c10d); returns the work object (work.wait() under a stream orders that stream after it)."""
    import torch.distributed as dist
    return dist.all_reduce(flat[lo:hi], group=group, async_op=True)


__all__ = ["env_rank_world", "shard", "tensor_buckets", "allreduce_bucket"]
