"""Numpy restatement of the PLDepth ranking samplers — TEST INFRASTRUCTURE (see oracle/__init__).

Restates, operation for operation and in the same floating-point types (NumPy 2.x / NEP 50
promotion, which is what the golden vectors were captured under):

  * ``sample_masked_rankings``        pldepth/data/sampling.py:131-145 (+ :111-122 per list)
  * Purely masked  (f=0.8, no score)  pldepth/data/sampling.py:147-150
  * Masked random  (f=1.5, Σ|Δg|)     pldepth/data/sampling.py:158-170
  * Thresholded    (f=1.5, Σ|Δg| − 1000·[eq])      pldepth/data/sampling.py:190-208
  * Information    (f=5, −Σ(g−e)²/e − 1000·[eq])   pldepth/data/sampling.py:218-239
  * ``get_depth_relation``            pldepth/data/depth_utils.py:5-21

Tie order. The reference sorts with ``np.argsort(x)[::-1]`` (default ``kind='quicksort'``, which
NumPy 2.x may dispatch to an unstable SIMD sort), so the order among EQUAL depths inside a list and
among EQUAL scores at the top-R cut is machine-dependent in the reference itself. This restatement
(and the HIP sampler, which must match it bit for bit) fixes it as a stable ascending argsort,
reversed: equal keys come out in DESCENDING original position. Tests against the reference's
golden vectors compare tie-insensitively (``canonical_lists``).

Draws. The reference calls ``np.random.randint(n_valid)`` once per list slot, list-major. Pass
``draws`` (int array [n_cand * L]) to replay a recorded sequence, or ``draws=None`` to consume the
global NumPy RNG in the same order (identical to the reference's stream for the same seed).
"""
import numpy as np

EQ_PENALTY = -1000
THRESHOLD = 0.03
FACTORS = {"pure": 0.8, "masked": 1.5, "thresh": 1.5, "info": 5}
_EPS32 = np.float32(1e-10)
_UP32 = np.float32(1 + THRESHOLD)        # python float cast to float32 (NEP 50 comparison)
_DOWN32 = np.float32(1 / (1 + THRESHOLD))


def n_candidates(R, strategy):
    """``int(batch_size * batch_size_factor)`` — sampling.py:55."""
    return int(R * FACTORS[strategy])


def get_depth_relation32(d1, d2):
    """Vectorised depth_utils.py:5-21 with threshold τ=0.03 on float32 inputs.

    ``(d1 + 1e-10) / (d2 + 1e-10)`` is evaluated in float32 (NEP 50: float32 scalar op Python
    float → float32) and compared with float32(1.03) / float32(1/1.03).
    """
    d1 = np.asarray(d1, np.float32)
    d2 = np.asarray(d2, np.float32)
    with np.errstate(divide="ignore", invalid="ignore"):
        r = (d1 + _EPS32) / (d2 + _EPS32)
    return np.where(r >= _UP32, 1, np.where(r <= _DOWN32, -1, 0)).astype(np.int8)


def pairwise_sum32(x):
    """NumPy's float32 ``add.reduce`` of a contiguous 1-D array: 0 + pairwise_sum(x).

    Restated so the HIP kernel can follow the same association (numpy/_core/src/umath/
    loops_utils.h.src ``pairwise_sum``: <8 sequential; ≤128 eight strided partials; else split at
    n/2 rounded down to a multiple of 8).
    """
    x = np.asarray(x, np.float32)

    def pw(a):
        n = a.size
        if n < 8:
            res = np.float32(-0.0)
            for v in a:
                res = np.float32(res + v)
            return res
        if n <= 128:
            r = [np.float32(v) for v in a[:8]]
            i = 8
            while i < n - (n % 8):
                for j in range(8):
                    r[j] = np.float32(r[j] + a[i + j])
                i += 8
            res = np.float32(np.float32(r[0] + r[1]) + np.float32(r[2] + r[3]))
            res = np.float32(res + np.float32(np.float32(r[4] + r[5]) + np.float32(r[6] + r[7])))
            while i < n:
                res = np.float32(res + a[i])
                i += 1
            return res
        n2 = n // 2
        n2 -= n2 % 8
        return np.float32(pw(a[:n2]) + pw(a[n2:]))

    return np.float32(np.float32(0.0) + pw(x))


def info_expected_list(gt, L):
    """``np.linspace(min(gt) + 0.001, max(gt), L + 1)[1:]`` in float32 (sampling.py:219-223)."""
    start = np.float32(np.float32(np.amin(gt)) + np.float32(0.001))
    stop = np.float32(np.amax(gt))
    return np.linspace(start, stop, L + 1)[1:]


def _sorted_desc_order(keys):
    """Row-wise stable ascending argsort, reversed (descending; ties → higher position first)."""
    return np.argsort(keys, axis=-1, kind="stable")[..., ::-1]


def sample_candidates(mask, gt, n_cand, L, draws=None):
    """sampling.py:111-145: n_cand lists of L masked pixels, each sorted by gt descending.

    Returns float32 [n_cand, L, 2] with column 0 = flat index ``row*W + col`` (float32, exact
    below 2**24) and column 1 = gt, plus the draws used (int64 [n_cand*L]).
    """
    H, W = gt.shape
    rows, cols = np.where(mask > 0)  # sampling.py:135, row-major order
    nvalid = rows.shape[0]
    if draws is None:
        draws = np.random.randint(nvalid, size=n_cand * L)
    draws = np.asarray(draws, np.int64).reshape(n_cand, L)
    if draws.size and (draws.min() < 0 or draws.max() >= nvalid):
        raise ValueError("draw out of range")
    r = rows[draws]
    c = cols[draws]  # x_scale = y_scale = 1 (mask and image share a shape on every caller)
    idx = (r * W + c).astype(np.float64)
    g = gt[r, c].astype(np.float64)
    order = _sorted_desc_order(g)
    out = np.empty((n_cand, L, 2), np.float32)
    out[:, :, 0] = np.take_along_axis(idx, order, axis=1)
    out[:, :, 1] = np.take_along_axis(g, order, axis=1)
    return out, draws.reshape(-1)


def score_candidates(cands, strategy, gt=None):
    """Per-list scores (float64 array) exactly as the reference accumulates them."""
    n_cand, L, _ = cands.shape
    g = cands[:, :, 1]  # float32 view, as result_matrix[i, :, 1]
    scores = np.zeros(n_cand, np.float64)
    if strategy == "pure":
        return scores
    if strategy in ("masked", "thresh"):
        diff = np.abs(g[:, :-1] - g[:, 1:])  # float32
        eq = get_depth_relation32(g[:, :-1], g[:, 1:]) == 0
        acc = np.zeros(n_cand, np.float32)
        for j in range(L - 1):  # sampling.py:199-206: penalty first, then the difference
            if strategy == "thresh":
                acc = np.where(eq[:, j], (acc + np.float32(EQ_PENALTY)).astype(np.float32), acc)
            acc = (acc + diff[:, j]).astype(np.float32)
        scores[:] = acc
        return scores
    if strategy == "info":
        e = info_expected_list(gt, L)
        terms = (np.square(g - e) / e).astype(np.float32)  # float32 elementwise
        for i in range(n_cand):
            scores[i] = -pairwise_sum32(terms[i])
        eq = get_depth_relation32(g[:, :-1], g[:, 1:]) == 0
        for j in range(L - 1):  # sampling.py:236-237, float64 accumulation
            scores = np.where(eq[:, j], scores + EQ_PENALTY, scores)
        return scores
    raise ValueError(strategy)


def sample_masked_point_batch(strategy, mask, gt, R, L, draws=None):
    """``<Strategy>.sample_masked_point_batch(image, mask, gt, R)`` → float32 [R', L, 2]."""
    n_cand = n_candidates(R, strategy)
    cands, used = sample_candidates(mask, gt, n_cand, L, draws)
    if strategy == "pure":
        return cands[:R], used
    scores = score_candidates(cands, strategy, gt)
    order = np.argsort(scores, kind="stable")[::-1][:R]
    return cands[order], used


def canonical_lists(out):
    """Tie-insensitive canonical form: within each list, sort (gt desc, idx asc); then order the
    lists lexicographically. Two sampler outputs that differ only in tie order compare equal."""
    out = np.asarray(out, np.float64)
    lists = []
    for lst in out:
        o = np.lexsort((lst[:, 0], -lst[:, 1]))
        lists.append(lst[o].reshape(-1))
    lists.sort(key=lambda v: tuple(v))
    return np.array(lists)
