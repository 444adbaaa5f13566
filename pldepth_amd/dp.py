"""Data-parallel plumbing: one process per GPU, torch.distributed ("nccl" = RCCL over xGMI on
ROCm, "gloo" on CPU for tests).

The reference trains on one device; the build shards HR-WSI-shaped minibatches:
rank r owns images [r*B, (r+1)*B) of the global batch (contiguous), draws its rankings and
drop-connect masks from Philox counters keyed by the GLOBAL image index (so results do not
depend on the GPU count), keeps BN statistics per replica (TF MirroredStrategy semantics) and
exchanges exactly one thing per step: the fp32 gradient, summed by all-reduce in reverse-order
buckets as the backward finalises them (``BucketSchedule``) and averaged inside the Adam kernel
(grad_scale = 1/world). ``ReplicaTrainer`` (trainer.py) drives both, eagerly and between the
segment graphs of its captured step.
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


class BucketSchedule(object):
    """Bucket boundaries of a flat gradient buffer that the backward finalises from the end
    towards offset 0 (engine.backward(grad_ready=...) reports 'grads[off:] are final').

    ready(off) returns the bucket (lo, hi) to exchange now — once at least `bucket_bytes` are
    pending, and always at off == 0 (the end of the backward) — or None. Over one backward the
    buckets tile [0, numel) exactly, in reverse order. ~8 MB buckets: large enough that each
    RCCL ring all-reduce runs at link rate over xGMI (7 x ~153 GB/s point-to-point links), small
    enough that the first one starts while most of the backward is still running."""

    def __init__(self, numel, bucket_bytes=8 << 20, elem_bytes=4):
        self.numel, self.bucket_bytes, self.elem_bytes = int(numel), int(bucket_bytes), elem_bytes
        self.reset()

    def reset(self):
        self.hi = self.numel

    def ready(self, off):
        pending = (self.hi - off) * self.elem_bytes
        if off < self.hi and (pending >= self.bucket_bytes or off == 0):
            bucket = (int(off), self.hi)
            self.hi = int(off)
            return bucket
        return None

    @property
    def done(self):
        return self.hi == 0


def allreduce_bucket(flat, lo, hi, group=None):
    """Async sum-all-reduce of flat[lo:hi] (ordered after the caller's current stream by
    c10d); returns the work object (work.wait() under a stream orders that stream after it)."""
    import torch.distributed as dist
    return dist.all_reduce(flat[lo:hi], group=group, async_op=True)


__all__ = ["env_rank_world", "shard", "BucketSchedule", "allreduce_bucket"]
