"""NumPy Philox4x32-10 and the counter layouts the HIP path keys its random streams with — TEST
INFRASTRUCTURE (see oracle/__init__).

The reference draws its random numbers from stateful generators that a GPU cannot replay: the
global NumPy RNG for the ranking sampler (pldepth/data/sampling.py:113, np.random.randint) and
TF's stateful dropout RNG for EfficientNet's drop-connect (Keras Dropout(noise_shape=(N,1,1,1)),
[3P] keras.applications.efficientnet). The build replaces both with counter-based Philox streams
keyed by (seed, step, global image, slot) — reproducible at any GPU count. The distributions are
the reference's (uniform integer in [0, n); keep with probability 1 - rate, scale 1/(1 - rate));
the bits are this build's own, so they are pinned here by a restatement of the generator (Salmon
et al., SC'11, Philox4x32 with 10 rounds; the Random123 constants) rather than by the reference.
"""
import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)
MASK32 = np.uint64(0xFFFFFFFF)


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised Philox4x32-10: counters (uint32 arrays), key (uint32 scalars) -> 4 uint32."""
    c0, c1, c2, c3 = (np.asarray(v, np.uint32).copy() for v in (c0, c1, c2, c3))
    k0, k1 = np.uint32(k0), np.uint32(k1)
    with np.errstate(over="ignore"):
        for _ in range(10):
            p0 = M0 * c0.astype(np.uint64)
            p1 = M1 * c2.astype(np.uint64)
            hi0, lo0 = (p0 >> np.uint64(32)).astype(np.uint32), (p0 & MASK32).astype(np.uint32)
            hi1, lo1 = (p1 >> np.uint64(32)).astype(np.uint32), (p1 & MASK32).astype(np.uint32)
            c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
            k0 = np.uint32(k0 + W0)
            k1 = np.uint32(k1 + W1)
    return c0, c1, c2, c3


def _split64(v):
    v = int(v) & 0xFFFFFFFFFFFFFFFF
    return np.uint32(v & 0xFFFFFFFF), np.uint32(v >> 32)


def sampler_draws(nvalid, n_cand, L, seed, step, image_offset=0):
    """pld_sampler_draw (csrc/sampler.hip draw_kernel): draw j of image b is
    floor(u32 * nvalid[b] / 2^32) with u32 = Philox(counter = (j, image_offset + b, step_lo,
    step_hi), key = seed).x. Returns int32 [B, n_cand, L]."""
    nvalid = np.asarray(nvalid, np.int64)
    B = nvalid.shape[0]
    per = n_cand * L
    slot = np.tile(np.arange(per, dtype=np.uint32), B)
    img = np.repeat(np.arange(B, dtype=np.uint32) + np.uint32(image_offset), per)
    s0, s1 = _split64(step)
    k0, k1 = _split64(seed)
    x, _, _, _ = philox4x32_10(slot, img, np.full_like(slot, s0), np.full_like(slot, s1), k0, k1)
    n = np.repeat(np.maximum(nvalid, 0).astype(np.uint64), per)
    d = (x.astype(np.uint64) * n) >> np.uint64(32)
    return d.astype(np.int32).reshape(B, n_cand, L)


def dropconnect_scales(n, rate, seed, step, layer, image_offset=0):
    """pld_dropconnect_scales (csrc/resample.hip dropconnect_kernel): per image i, u = (x >> 8) /
    2^24 with x = Philox(counter = (layer, image_offset + i, step_lo, step_hi ^ 0x5D0C), key =
    seed).x; scale = 1/(1 - rate) in float32 if u >= rate else 0 (TF2 dropout: keep_mask =
    uniform >= rate, x * scale). Returns float32 [n]."""
    i = np.arange(n, dtype=np.uint32) + np.uint32(image_offset)
    s0, s1 = _split64(step)
    k0, k1 = _split64(seed)
    x, _, _, _ = philox4x32_10(np.full_like(i, layer), i, np.full_like(i, s0),
                               np.full_like(i, s1 ^ np.uint32(0x5D0C)), k0, k1)
    u = (x >> np.uint32(8)).astype(np.float32) * np.float32(1.0 / 16777216.0)
    keep = u >= np.float32(rate)
    return np.where(keep, np.float32(1.0) / (np.float32(1.0) - np.float32(rate)),
                    np.float32(0.0)).astype(np.float32)
