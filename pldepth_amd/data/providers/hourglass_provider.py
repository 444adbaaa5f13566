"""Training / validation batch provider (mirrors pldepth/data/providers/hourglass_provider.py).

The reference builds a tf.data pipeline: zip(img, mask, gt) -> random joint horizontal flip ->
shuffle(1024) -> tf.numpy_function(sampler) per image -> batch(drop_remainder) -> prefetch ->
repeat (provide_train_dataset, :29-62), and pre-generates validation rankings once with the
Thresholded sampler (provide_val_dataset / generate_validation_rankings, :64-73, :179-193).

Here the datasets are in-memory arrays (images [N,H,W,3] in [0,1], gts [N,H,W], masks [N,H,W]);
flips and shuffling are host index work, and the rankings of a whole batch come from ONE GPU
sampler launch (Philox draws keyed by seed / batch counter / image position) instead of a
per-image Python call under the GIL. Batches are (x [B,H,W,3], y [B,R,L,2]) device tensors.
"""
import numpy as np
import torch

from ..sampling import ThresholdedMaskedRandomSamplingStrategy


class HourglassLargeScaleDataProvider(object):
    def __init__(self, model_params, train_consistency_masks, val_consistency_masks,
                 loss_type=None, augmentation=False, sampling_eq_threshold=0.03, bs_factor=5,
                 seed=0):
        self.model_params = model_params
        self.train_consistency_masks = np.asarray(train_consistency_masks, np.float32)
        self.val_consistency_masks = (None if val_consistency_masks is None else
                                      np.asarray(val_consistency_masks, np.float32))
        self.random_sampler = ThresholdedMaskedRandomSamplingStrategy(model_params,
                                                                     sampling_eq_threshold)
        self.val_random_sampler = ThresholdedMaskedRandomSamplingStrategy(model_params)
        self.augmentation = augmentation
        self.loss_type = loss_type
        self.bs_factor = bs_factor
        self.seed = seed

    def provide_train_dataset(self, base_ds, base_ds_gts=None):
        return _TrainIterable(self, np.asarray(base_ds, np.float32),
                              np.asarray(base_ds_gts, np.float32))

    def provide_val_dataset(self, base_ds, base_ds_gts=None):
        imgs = np.asarray(base_ds, np.float32)
        gts = np.asarray(base_ds_gts, np.float32)
        B = self.model_params.get_parameter("batch_size")
        R = self.model_params.get_parameter("val_rankings_per_img")
        dev = torch.device("cuda", torch.cuda.current_device())
        batches = []
        for i in range(0, len(imgs) - B + 1, B):  # batch(drop_remainder=True) + cache()
            y = self.val_random_sampler.sample_batch_gpu(
                torch.from_numpy(gts[i:i + B]).to(dev),
                torch.from_numpy(self.val_consistency_masks[i:i + B]).to(dev), R,
                seed=self.seed + 7919, step=0, image_offset=i)
            batches.append((torch.from_numpy(imgs[i:i + B]).to(dev), y))
        return batches


class _TrainIterable(object):
    def __init__(self, prov, imgs, gts):
        self.p, self.imgs, self.gts = prov, imgs, gts
        self.masks = prov.train_consistency_masks

    def __iter__(self):
        p = self.p
        B = p.model_params.get_parameter("batch_size")
        R = p.model_params.get_parameter("rankings_per_image")
        strategy = p.model_params.get_parameter("sampling_strategy") or p.random_sampler
        rng = np.random.default_rng(p.seed)
        dev = torch.device("cuda", torch.cuda.current_device())
        n = len(self.imgs)
        step = 0
        while True:  # repeat()
            order = rng.permutation(n)
            for i in range(0, n - B + 1, B):
                idx = order[i:i + B]
                x, g, m = self.imgs[idx], self.gts[idx], self.masks[idx]
                if p.augmentation:  # joint random horizontal flip, p = 0.5 (:35-49)
                    flip = rng.random(B) > 0.5
                    x = np.where(flip[:, None, None, None], x[:, :, ::-1], x)
                    g = np.where(flip[:, None, None], g[:, :, ::-1], g)
                    m = np.where(flip[:, None, None], m[:, :, ::-1], m)
                gd = torch.from_numpy(np.ascontiguousarray(g)).to(dev)
                md = torch.from_numpy(np.ascontiguousarray(m)).to(dev)
                y = strategy.sample_batch_gpu(gd, md, R, seed=p.seed, step=step, image_offset=0)
                step += 1
                yield torch.from_numpy(np.ascontiguousarray(x)).to(dev), y
