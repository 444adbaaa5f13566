"""Ranking samplers (mirrors pldepth/data/sampling.py) backed by the GPU sampler.

Same class names, constructors and per-image entry point as the reference:
``Strategy(model_params).sample_masked_point_batch(image, mask, gt, batch_size)`` ->
float32 [R', L, 2] (flat pixel index row*W+col, depth), lists sorted by depth descending, the
best-scoring R kept. Like the reference, the per-image call consumes the global NumPy RNG —
``np.random.randint(n_valid)`` once per list slot, list-major (sampling.py:113) — and ships the
draws to pld_sampler_rank, so a seeded run reproduces the reference's rankings (ties aside,
which the reference itself orders machine-dependently).

The batched GPU path (``sample_batch_gpu``) keeps draws on the device (Philox counter keyed by
seed/step/image: independent of the GPU count) and is what the training step uses.
"""
import numpy as np
import torch

from .. import kernels as K
from .depth_utils import get_depth_relation  # noqa: F401  (re-exported like the reference)


class SamplingStrategy(object):
    NAME = None

    def __init__(self, model_params):
        self.num_points_per_sample = model_params.get_parameter("ranking_size")

    @property
    def num_points_per_sample(self):
        return self._num_points_per_sample

    @num_points_per_sample.setter
    def num_points_per_sample(self, value):
        self._num_points_per_sample = value

    def __str__(self):
        return "{}(num_points_per_sample={})".format(self.__class__.__name__,
                                                    self._num_points_per_sample)

    # ---------------------------------------------------------------- GPU batch entry
    def sample_batch_gpu(self, gt, mask, batch_size, seed=0, step=0, image_offset=0,
                         draws=None):
        """gt, mask: [B,H,W] device tensors -> [B, R', L, 2] device tensor (Philox draws, or
        explicit draws [B, n_cand, L] int32)."""
        B, H, W = gt.shape
        L = self._num_points_per_sample
        dev = gt.device
        nc = K.sampler_candidates(batch_size, self.NAME)
        r_out = nc if self.NAME == "pure" else batch_size
        vi = torch.empty(B, H * W, dtype=torch.int32, device=dev)
        nv = torch.empty(B, dtype=torch.int32, device=dev)
        mm = torch.empty(B, 2, device=dev)
        K.sampler_compact(mask.contiguous(), gt.contiguous(), vi, nv, mm)
        if draws is None:
            draws = torch.empty(B, nc, L, dtype=torch.int32, device=dev)
            K.sampler_draw(nv, nc, L, seed, step, image_offset, draws)
        out = torch.empty(B, r_out, L, 2, device=dev)
        K.sampler_rank(gt.contiguous(), vi, nv, mm, draws.contiguous(), batch_size, L,
                       self.NAME, out)
        return out

    # ---------------------------------------------------------------- reference entry
    def sample_masked_point_batch(self, image, mask, gt, batch_size, batch_size_factor=None):
        if batch_size_factor is not None and batch_size_factor != self.FACTOR:
            raise NotImplementedError("non-default batch_size_factor")
        mask = np.asarray(mask, np.float32)
        gt = np.asarray(gt, np.float32)
        if mask.shape != gt.shape[:2]:
            raise NotImplementedError("mask and gt must share the image's spatial shape")
        L = self._num_points_per_sample
        nc = K.sampler_candidates(batch_size, self.NAME)
        n_valid = int((mask > 0).sum())
        draws = np.random.randint(n_valid, size=nc * L).astype(np.int32)  # sampling.py:113
        dev = torch.device("cuda", torch.cuda.current_device())
        out = self.sample_batch_gpu(torch.from_numpy(gt)[None].to(dev),
                                    torch.from_numpy(mask)[None].to(dev), batch_size,
                                    draws=torch.from_numpy(draws).view(1, nc, L).to(dev))
        return out[0].cpu().numpy()


class PurelyMaskedRandomSamplingStrategy(SamplingStrategy):
    """sampling.py:106-150: floor(0.8 R) lists, no scoring."""
    NAME, FACTOR = "pure", 0.8


class MaskedRandomSamplingStrategy(SamplingStrategy):
    """sampling.py:153-170: 1.5 R candidates scored by the sum of adjacent depth gaps."""
    NAME, FACTOR = "masked", 1.5


class ThresholdedMaskedRandomSamplingStrategy(SamplingStrategy):
    """sampling.py:172-208: as Masked, -1000 per adjacent pair within tau = 0.03."""
    NAME, FACTOR = "thresh", 1.5

    def __init__(self, model_params, threshold=0.03, equality_penalty=-1000):
        super().__init__(model_params)
        if threshold != 0.03 or equality_penalty != -1000:
            raise NotImplementedError("the HIP sampler is built for tau=0.03, penalty=-1000")
        self.threshold, self.equality_penalty = threshold, equality_penalty


class InformationScoreBasedSampling(SamplingStrategy):
    """sampling.py:211-242: 5 R candidates scored by -sum (g - e)^2 / e against an evenly spaced
    expected list, -1000 per near-equal adjacent pair (the PLDepth.py default)."""
    NAME, FACTOR = "info", 5

    def __init__(self, model_params, threshold=0.03, equality_penalty=-1000):
        super().__init__(model_params)
        if threshold != 0.03 or equality_penalty != -1000:
            raise NotImplementedError("the HIP sampler is built for tau=0.03, penalty=-1000")
        self.threshold, self.equality_penalty = threshold, equality_penalty

    def __str__(self):
        return "{}(num_points_per_sample={}, threshold={})".format(
            self.__class__.__name__, self._num_points_per_sample, self.threshold)
