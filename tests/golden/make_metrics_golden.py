"""Generate test-pass metric golden vectors from the REFERENCE functions (container-only script).

Runs the reference's ``ordinal_error`` (pldepth/active_learning/metrics.py:60-70) and ``calc_d``
(metrics.py:92-109) on seeded synthetic predictions / depth maps and writes the inputs, the
pixel indices those calls drew from numpy's global RNG, and the results to
``metrics_golden.npz``. Only arrays are written; no reference source is copied.

metrics.py imports OpenCV (``cv2``) and ``preprocess_utils`` (which imports cv2); OpenCV is not
installed here. A placeholder ``cv2`` module is registered whose only callable, ``normalize``,
implements NORM_MINMAX by OpenCV's documented formula — so ``calc_d``'s normalisation step is
this script's restatement (unpinned), while its sampling, sorting and DCG logic, and all of
``ordinal_error``, are the reference's own. scipy (cKDTree, imported at module level) is real.

Run:  python tests/golden/make_metrics_golden.py
"""
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"


def _cv2_stub():
    m = types.ModuleType("cv2")
    m.NORM_MINMAX = 32

    def normalize(src, dst, alpha, beta, norm_type):
        assert norm_type == m.NORM_MINMAX and dst is None
        src = np.asarray(src, np.float32)
        dmin, dmax = min(alpha, beta), max(alpha, beta)
        smin, smax = float(src.min()), float(src.max())
        scale = (dmax - dmin) * (1.0 / (smax - smin) if smax - smin > np.finfo(float).eps else 0)
        shift = dmin - smin * scale
        return (src.astype(np.float64) * scale + shift).astype(np.float32)

    m.normalize = normalize
    return m


def _import_reference_metrics():
    sys.modules["cv2"] = _cv2_stub()
    sys.path.insert(0, REF)
    from pldepth.active_learning import metrics  # noqa: E402
    assert metrics.__file__.startswith(REF), metrics.__file__
    return metrics


def _depth(h, w, rng):
    yy, xx = np.meshgrid(np.linspace(0, 1, h), np.linspace(0, 1, w), indexing="ij")
    f = np.sin(2 * np.pi * rng.uniform(0.5, 2) * yy + rng.uniform(0, 6)) * \
        np.cos(2 * np.pi * rng.uniform(0.5, 2) * xx + rng.uniform(0, 6))
    f = (f - f.min()) / (f.max() - f.min())
    return (np.round(255 * f) / 255).astype(np.float32)[..., None]  # 8-bit ties, [H, W, 1]


def main():
    M = _import_reference_metrics()
    rng = np.random.default_rng(2024)
    out = {}
    # ordinal_error: (H, W, num) incl. every pixel used once (2 num = H W)
    for c, (h, w, num) in enumerate([(48, 40, 500), (32, 32, 512), (20, 30, 7)]):
        op = rng.standard_normal((h, w, 1)).astype(np.float32)
        op[::3, ::5] = op[1, 1]  # predicted ties
        gt = _depth(h, w, rng)
        err = M.ordinal_error(op, gt, imsize=(h, w), num=num)
        np.random.seed(10)  # the indices that call drew
        idx = np.random.choice(list(range(h * w)), num * 2, replace=False)
        out[f"ord{c}_op"], out[f"ord{c}_gt"] = op, gt
        out[f"ord{c}_idx"] = idx.astype(np.int32)
        out[f"ord{c}_num"] = np.int32(num)
        out[f"ord{c}_err"] = np.float64(err)
    # calc_d: (H, W, list_size)
    for c, (h, w, ls) in enumerate([(24, 24, 200), (40, 36, 200), (16, 20, 64)]):
        op = (rng.standard_normal((h, w, 1)) * 3 + 1).astype(np.float32)
        gt = _depth(h, w, rng)
        d = M.calc_d(op, gt, imsize=(h, w), list_size=ls)
        np.random.seed(69)
        ids = np.random.choice(np.arange(h * w), size=ls, replace=False)
        out[f"dcg{c}_op"], out[f"dcg{c}_gt"] = op, gt
        out[f"dcg{c}_ids"] = ids.astype(np.int32)
        out[f"dcg{c}_d"] = np.float64(d)
    np.savez_compressed(os.path.join(HERE, "metrics_golden.npz"), **out)
    print({k: float(v) for k, v in out.items() if k.endswith(("_err", "_d"))})


if __name__ == "__main__":
    main()
