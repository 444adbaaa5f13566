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


def init_group(backend, rank, world, device=None, timeout_s=600):
    """torch.distributed.init_process_group with a bound: the rendezvous and every later
    collective raise after `timeout_s` instead of waiting forever on a rank that never arrives or
    has died. "nccl" (RCCL) binds the group to `device` and turns on the watchdog's
    asynchronous error handling, which aborts a collective stuck past the timeout; "gloo" raises
    from the blocked call itself (or at once when a peer's socket closes)."""
    import datetime
    import torch.distributed as dist
    td = datetime.timedelta(seconds=timeout_s)
    if backend == "nccl":
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=device, timeout=td)
    else:
        dist.init_process_group(backend, rank=rank, world_size=world, timeout=td)
    return dist.group.WORLD


def rccl_version():
    """"major.minor.patch" of the RCCL library torch.distributed's nccl backend loaded (None when
    torch has no nccl/RCCL build)."""
    try:
        import torch
        v = torch.cuda.nccl.version()
    except Exception:
        return None
    return ".".join(str(x) for x in v) if isinstance(v, tuple) else str(v)


def replica_checksum(buf):
    """Two int64 checksums of a flat fp32 buffer's BIT patterns: their plain sum and a sum
    weighted by position (1 + i mod 1021), so equal checksums mean equal buffers up to a
    collision, not merely equal values in another order. Wraps modulo 2^64 (deterministic)."""
    import torch
    bits = buf.detach().reshape(-1).view(torch.int32).to(torch.int64)
    w = (torch.arange(bits.numel(), device=bits.device, dtype=torch.int64) % 1021) + 1
    return torch.stack([bits.sum(), (bits * w).sum()])


def replicas_identical(buf, group=None):
    """After data-parallel steps every replica must hold the same parameters bit for bit (they
    apply the same all-reduced gradient to the same weights). All-reduces MIN and MAX of each
    rank's replica_checksum; returns (identical, {min, max})."""
    import torch.distributed as dist
    c = replica_checksum(buf)
    lo, hi = c.clone(), c.clone()
    dist.all_reduce(lo, op=dist.ReduceOp.MIN, group=group)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX, group=group)
    lo, hi = lo.tolist(), hi.tolist()
    return lo == hi, {"min": lo, "max": hi}


def exit_on_failure(fn, world):
    """Run fn(); in a multi-rank job an exception (a dead peer, a collective past its timeout)
    ends THIS rank at once with a non-zero status instead of leaving it blocked in a later
    collective or in process-group teardown; the launcher then stops the remaining ranks."""
    import sys
    import traceback
    try:
        return fn()
    except BaseException as e:  # noqa: B902  (SystemExit included: keep its code)
        if world <= 1:
            raise
        code = e.code if isinstance(e, SystemExit) and isinstance(e.code, int) and e.code else 1
        rank = os.environ.get("RANK", "?")
        print(f"[rank {rank}] failed: {type(e).__name__}: {e}", file=sys.stderr, flush=True)
        traceback.print_exc(file=sys.stderr)
        sys.stderr.flush()
        os._exit(code)


__all__ = ["env_rank_world", "shard", "tensor_buckets", "allreduce_bucket", "init_group",
           "rccl_version", "replica_checksum", "replicas_identical", "exit_on_failure"]
