"""PLDepth training entry point (mirrors pldepth/PLDepth.py:28-209 — same click flags).

    python -m pldepth_amd.PLDepth --model_name ff_effnet --batch_size 32 --ranking_size 5 \\
        --rankings_per_image 100 --epochs 2 --ds_size 256 --input_size 448

Differences from the reference driver, all outside the accelerated path:
  * data: ``--hr_wsi_path`` reads the HR-WSI tree (pldepth_amd.data.dao.hr_wsi: host decode, GPU
    resize); ``--data_npz`` loads in-memory arrays (imgs [N,H,W,3] in [0,1], gts [N,H,W],
    masks [N,H,W]); without either a seeded synthetic HR-WSI-shaped set is generated;
  * no wandb / mlflow: metrics go to stdout and ``--log_jsonl``;
  * ``--input_size`` (the reference hard-codes 224 here and 448 in run_scripts/test_sampling.py).
Everything per step — sampling, forward, ListMLE, backward, Adam-AMSGrad — runs on the GPU.
"""
import json
import os
import time

import click
import numpy as np

from .losses.losses_meta import DepthLossType
from .losses.nll_loss import HourglassNegativeLogLikelihood
from .models.models_meta import ModelParameters, get_model_type_by_name
from .models.PLDepthNet import get_pl_depth_net
from .optimizers import Adam
from .data.sampling import (InformationScoreBasedSampling, PurelyMaskedRandomSamplingStrategy,
                            ThresholdedMaskedRandomSamplingStrategy)
from .data.providers.hourglass_provider import HourglassLargeScaleDataProvider
from .util.training_utils import LearningRateLoggingCallback, SGDRScheduler, TerminateOnNaN
from .active_learning.metrics import calc_err, dcg_metric


def synthetic_hrwsi(n, h, w, seed=0):
    """Seeded stand-in for HR-WSI: U[0,1) RGB, smooth 8-bit depth, Bernoulli(0.9) masks."""
    rng = np.random.default_rng(seed)
    imgs = rng.random((n, h, w, 3), dtype=np.float32)
    yy, xx = np.meshgrid(np.linspace(0, 1, h), np.linspace(0, 1, w), indexing="ij")
    gts = np.empty((n, h, w), np.float32)
    for i in range(n):
        f = np.zeros((h, w))
        for _ in range(4):
            fy, fx = rng.uniform(0.3, 3.0, 2)
            ph = rng.uniform(0, 2 * np.pi, 2)
            f += rng.uniform(0.2, 1.0) * np.sin(2 * np.pi * fy * yy + ph[0]) * \
                np.cos(2 * np.pi * fx * xx + ph[1])
        f = (f - f.min()) / (f.max() - f.min())
        gts[i] = np.round(255 * f) / 255
    masks = (rng.random((n, h, w)) < 0.9).astype(np.float32)
    return imgs, gts, masks


class JSONLLogger(object):
    def __init__(self, path):
        self.path = path
        self.t0 = time.time()

    def set_model(self, model):
        self.model = model

    def on_batch_end(self, batch, logs=None):
        if self.path:
            with open(self.path, "a") as f:
                f.write(json.dumps({"t": time.time() - self.t0, "batch": batch,
                                    "lr": self.model.optimizer.lr, **(logs or {})}) + "\n")


@click.command()
@click.option('--model_name', default='ff_effnet', help='Backbone model',
              type=click.Choice(['ff_redweb', 'ff_effnet'], case_sensitive=False))
@click.option('--epochs', default=50)
@click.option('--batch_size', default=4)
@click.option('--seed', default=0)
@click.option('--ranking_size', default=3, help='Number of elements per training ranking')
@click.option('--rankings_per_image', default=100, help='Number of rankings per image')
@click.option('--initial_lr', default=0.01, type=click.FLOAT)
@click.option('--equality_threshold', default=0.03, type=click.FLOAT)
@click.option('--model_checkpoints', default=False, type=click.BOOL)
@click.option('--load_model_path', default='')
@click.option('--augmentation', default=True, type=click.BOOL)
@click.option('--warmup', default=0, type=click.INT)
@click.option('--sampling_type', default=1, type=click.INT)
@click.option('--lr_multi', default=0.25, type=click.FLOAT)
@click.option('--ds_size', default=None, type=click.INT)
@click.option('--input_size', default=224, type=click.INT)
@click.option('--data_npz', default='', help='npz with imgs/gts/masks arrays')
@click.option('--hr_wsi_path', default='', help='HR-WSI root ({train,val}/{imgs,gts,valid_masks})')
@click.option('--save_path', default='', help='save weights after training (.h5: Keras HDF5, '
              'else .npz) and the whole model as <stem>_model.h5')
@click.option('--log_jsonl', default='', help='per-batch metrics file')
def perform_pldepth_experiment(model_name, epochs, batch_size, seed, ranking_size,
                               rankings_per_image, initial_lr, equality_threshold,
                               model_checkpoints, load_model_path, augmentation, warmup,
                               sampling_type, lr_multi, ds_size, input_size, data_npz, save_path,
                               log_jsonl, hr_wsi_path=''):
    np.random.seed(seed)
    model_params = ModelParameters()
    model_params.set_parameter("model_type", get_model_type_by_name(model_name))
    model_params.set_parameter("epochs", epochs)
    model_params.set_parameter("ranking_size", ranking_size)
    model_params.set_parameter("rankings_per_image", rankings_per_image)
    model_params.set_parameter("val_rankings_per_img", rankings_per_image)
    model_params.set_parameter("batch_size", batch_size)
    model_params.set_parameter("seed", seed)
    model_params.set_parameter("equality_threshold", equality_threshold)
    model_params.set_parameter("loss_type", DepthLossType.NLL)
    model_params.set_parameter("augmentation", augmentation)
    model_params.set_parameter("warmup", warmup)
    if sampling_type == 0:
        strategy = ThresholdedMaskedRandomSamplingStrategy(model_params)
    elif sampling_type == 1:
        strategy = InformationScoreBasedSampling(model_params)
    elif sampling_type == 3:
        strategy = PurelyMaskedRandomSamplingStrategy(model_params)
    else:
        print("wrong selection of sampling type")
        return 13
    model_params.set_parameter("sampling_strategy", strategy)
    shape = [input_size, input_size, 3]
    model, preprocess_fn = get_pl_depth_net(model_params, shape)

    # eval split for the test pass (PLDepth.py:151,184-192: HR-WSI 'val', first 250 images)
    eval_imgs = eval_gts = None
    if hr_wsi_path:  # PLDepth.py:139-151: HR-WSI train split, decoded + resized (dao/hr_wsi.py)
        from .data.dao.hr_wsi import HRWSITFDataAccessObject
        dao = HRWSITFDataAccessObject(hr_wsi_path, shape, seed)
        imgs, gts, masks = dao.get_training_dataset(size=ds_size)
        gts = gts[..., 0]
        eval_imgs, eval_gts, _ = dao.get_validation_dataset()
        eval_imgs, eval_gts = eval_imgs[:250], eval_gts[:250, ..., 0]
    elif data_npz:
        with np.load(data_npz, allow_pickle=False) as z:
            imgs, gts, masks = z["imgs"], z["gts"], z["masks"]
            if "val_imgs" in z.files:
                eval_imgs, eval_gts = z["val_imgs"][:250], z["val_gts"][:250]
    else:
        imgs, gts, masks = synthetic_hrwsi(ds_size or 8 * batch_size, input_size, input_size,
                                           seed)
        n_eval = min(250, max(batch_size, len(imgs) // 15))
        eval_imgs, eval_gts, _ = synthetic_hrwsi(n_eval, input_size, input_size, seed + 1)
    ds_size = len(imgs)
    n_val = ds_size // 15
    steps_per_epoch = max(1, int((ds_size * 14 / 15) / batch_size))  # PLDepth.py:120
    schedule = SGDRScheduler(min_lr=initial_lr * (1 / lr_multi), max_lr=initial_lr,
                             steps_per_epoch=steps_per_epoch, lr_decay=0.9, cycle_length=epochs,
                             mult_factor=1)
    loss_fn = HourglassNegativeLogLikelihood(ranking_size=ranking_size, batch_size=batch_size)
    model.compile(loss=loss_fn, optimizer=Adam(learning_rate=initial_lr, amsgrad=True))
    if load_model_path:
        model.load_weights(load_model_path)
    provider = HourglassLargeScaleDataProvider(model_params, masks[n_val:], masks[:n_val],
                                               augmentation=augmentation, seed=seed)
    train_ds = provider.provide_train_dataset(preprocess_fn(imgs[n_val:]), gts[n_val:])
    val_ds = (provider.provide_val_dataset(preprocess_fn(imgs[:n_val]), gts[:n_val])
              if n_val >= batch_size else None)
    callbacks = [TerminateOnNaN(), schedule, LearningRateLoggingCallback(), JSONLLogger(log_jsonl)]
    if model_checkpoints:  # tracking_utils.py:21-30 (best val_loss -> Keras .h5 model file)
        from .util.env import get_config
        from .util.tracking_utils import construct_model_checkpoint_callback
        callbacks.append(construct_model_checkpoint_callback(get_config(), model_name, 1))
    model.fit(x=train_ds, epochs=epochs, steps_per_epoch=steps_per_epoch, callbacks=callbacks,
              validation_data=val_ds, verbose=1)
    if save_path:  # PLDepth.py:180-181: weights, plus the whole model as .h5
        model.save_weights(save_path)
        model.save(os.path.splitext(save_path)[0] + "_model.h5")
    # test pass (PLDepth.py:183-192): ordinal error and nDCG@200 on the first 250 images of the
    # held-out eval split, on the GPU (pldepth_amd.active_learning.metrics). Like the reference,
    # the images go in raw (no preprocess_fn: PLDepth.py:187-191 calls calc_err / dcg_metric on
    # the DAO's [0,1] images; for ff_effnet preprocessing is the identity anyway). The
    # reference's pair / list draws need >= 10,000 and >= 224*224 pixels per image.
    if eval_imgs is None:
        print("no eval split (--data_npz without val_imgs/val_gts): test pass skipped")
        return 0
    test_img, test_gt = eval_imgs, eval_gts
    if len(test_img) and input_size * input_size >= 2 * 5000:
        err = calc_err(model, test_img, test_gt[..., None], img_size=(input_size, input_size))
        print(f"test_error {err:.6f}")
    if len(test_img) and input_size >= 224:
        print(f"ndcg_200 {dcg_metric(model, test_img, test_gt[..., None], list_size=200):.6f}")
    return 0


if __name__ == "__main__":
    perform_pldepth_experiment()
