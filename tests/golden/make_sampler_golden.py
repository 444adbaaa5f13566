"""Generate sampler golden vectors from the REFERENCE numpy sampler (container-only script).

This script is the only place that imports the reference, and it runs only in the build container
(``/root/reference`` does not exist on the GPU box). It produces ``sampler_golden.npz`` next to
itself: inputs (8-bit gt codes, validity mask), the exact ``np.random.randint`` draw sequence the
reference consumed, and the reference outputs. No reference source or bytecode is copied: only
arrays are written.

Reference code exercised (read-only):
  * ``pldepth/data/sampling.py:111-122`` ``sample_single_masked_ranking``
  * ``pldepth/data/sampling.py:131-150`` ``sample_masked_rankings`` / Purely masked (f=0.8)
  * ``pldepth/data/sampling.py:158-170`` ``MaskedRandomSamplingStrategy`` (f=1.5)
  * ``pldepth/data/sampling.py:190-208`` ``ThresholdedMaskedRandomSamplingStrategy`` (f=1.5)
  * ``pldepth/data/sampling.py:218-239`` ``InformationScoreBasedSampling`` (f=5)
  * ``pldepth/data/depth_utils.py:5-21`` ``get_depth_relation``

``pldepth/data/depth_utils.py:1-2`` imports TensorFlow at module level (used only by
``get_depth_relation_tf``, which the sampler never calls); TF is not installed here, so an empty
placeholder module object (carrying only a `float32` name, read by a default argument at
definition time) is registered under that name before the import. Nothing of TF is
executed by the sampler.

Run:  python tests/golden/make_sampler_golden.py
"""
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"


def _import_reference_sampling():
    for name in ("tensorflow", "tensorflow.python", "tensorflow.python.keras",
                 "tensorflow.python.keras.backend"):
        sys.modules.setdefault(name, types.ModuleType(name))
    # `get_depth_relation_tf`'s default argument reads `tf.float32` at definition time
    sys.modules["tensorflow"].float32 = "float32"
    # the reference package is named `pldepth`; make sure nothing else shadows it
    sys.path.insert(0, REF)
    from pldepth.data import sampling, depth_utils  # noqa: E402
    assert sampling.__file__.startswith(REF), sampling.__file__
    return sampling, depth_utils


class _Params:
    def __init__(self, ranking_size):
        self.p = {"ranking_size": ranking_size, "downscaling_factor": 1}

    def get_parameter(self, name, default=None):
        return self.p.get(name, default)


def synthetic_gt_mask(h, w, seed):
    """Smooth 8-bit-quantised depth field + Bernoulli(0.9) mask."""
    rng = np.random.default_rng(seed)
    yy, xx = np.meshgrid(np.linspace(0, 1, h), np.linspace(0, 1, w), indexing="ij")
    field = np.zeros((h, w))
    for _ in range(6):
        fy, fx = rng.uniform(0.3, 3.0, 2)
        ph = rng.uniform(0, 2 * np.pi, 2)
        field += rng.uniform(0.2, 1.0) * np.sin(2 * np.pi * fy * yy + ph[0]) * np.cos(2 * np.pi * fx * xx + ph[1])
    field = (field - field.min()) / (field.max() - field.min())
    codes = np.round(255 * field).astype(np.uint8)
    mask = rng.random((h, w)) < 0.9
    return codes, mask


def gt_from_codes(codes):
    return codes.astype(np.float32) / np.float32(255.0)


def main():
    sampling, depth_utils = _import_reference_sampling()
    strategies = {
        "thresh": lambda p: sampling.ThresholdedMaskedRandomSamplingStrategy(p),
        "info": lambda p: sampling.InformationScoreBasedSampling(p),
        "pure": lambda p: sampling.PurelyMaskedRandomSamplingStrategy(p),
        "masked": lambda p: sampling.MaskedRandomSamplingStrategy(p),
    }
    # (H, W, L, R) — the BASELINE configs' sampler shapes, R reduced for the L=64 case to keep
    # the fixture small (the algorithm is per-candidate; R only sets how many are kept).
    configs = [(224, 224, 2, 100), (448, 448, 5, 100), (96, 128, 64, 12), (64, 64, 3, 40)]
    out = {}
    orig_randint = np.random.randint
    for ci, (h, w, L, R) in enumerate(configs):
        codes, mask = synthetic_gt_mask(h, w, seed=100 + ci)
        gt = gt_from_codes(codes)
        out[f"c{ci}_codes"] = codes
        out[f"c{ci}_mask"] = np.packbits(mask)
        out[f"c{ci}_shape"] = np.array([h, w, L, R], dtype=np.int64)
        image = np.zeros((h, w, 3), np.float32)
        maskf = mask.astype(np.float32)
        for sname, ctor in strategies.items():
            strat = ctor(_Params(L))
            draws = []

            def rec(*a, **k):
                v = orig_randint(*a, **k)
                draws.append(int(v))
                return v

            np.random.seed(1000 * ci + len(sname))
            np.random.randint = rec
            try:
                res = strat.sample_masked_point_batch(image, maskf, gt, R)
            finally:
                np.random.randint = orig_randint
            out[f"c{ci}_{sname}_draws"] = np.asarray(draws, dtype=np.int32)
            out[f"c{ci}_{sname}_out"] = np.asarray(res, dtype=np.float32)
            print(f"cfg{ci} {h}x{w} L={L} R={R} {sname}: draws={len(draws)} out={res.shape}")

    # get_depth_relation known answers at and around the tau boundary (float32 scalars, NumPy 2.x
    # NEP-50 promotion, as the sampler calls it with float32 list entries)
    rng = np.random.default_rng(7)
    d1 = np.concatenate([rng.random(2000), [0.0, 0.0, 1 / 255, 0.5]]).astype(np.float32)
    d2 = (d1 * rng.choice([1.0, 1.03, 1 / 1.03, 1.0299, 1.0301, 0.97], d1.size)).astype(np.float32)
    d2[-4:] = np.array([0.0, 0.5, 0.0, 0.5], np.float32)
    rel = np.array([depth_utils.get_depth_relation(a, b, 0.03) for a, b in zip(d1, d2)], np.int8)
    out["rel_d1"], out["rel_d2"], out["rel_out"] = d1, d2, rel
    np.savez_compressed(os.path.join(HERE, "sampler_golden.npz"), **out)
    print("wrote", os.path.join(HERE, "sampler_golden.npz"))


if __name__ == "__main__":
    main()
