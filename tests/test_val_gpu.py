"""the validation pass — val-ranking pre-generation and Keras' val_loss.

Reference: pldepth/data/providers/hourglass_provider.py:64-73 (provide_val_dataset: rankings
drawn once per val image by the Thresholded sampler, batched with drop_remainder and cached) and
Keras fit(validation_data=...) as PLDepth.py:144-149 drives it: after each epoch, val_loss = the
mean over the val batches of the loss, with every BN on its moving statistics.

Checked here against the oracle: the cached val rankings bit-exactly (oracle/sampler.py fed the
Philox draws of oracle/philox.py for (seed + 7919, step 0, image index)), and fit's val_loss
(oracle/effnet.py inference-mode forward + oracle/listmle.py on the post-fit weights).
"""
import numpy as np
import pytest
import torch

from oracle import effnet as OE
from oracle import listmle as LM
from oracle import philox as PX
from oracle import sampler as S
from pldepth_amd.data.providers.hourglass_provider import HourglassLargeScaleDataProvider
from pldepth_amd.data.sampling import InformationScoreBasedSampling
from pldepth_amd.losses.losses_meta import DepthLossType
from pldepth_amd.losses.nll_loss import HourglassNegativeLogLikelihood
from pldepth_amd.models.models_meta import ModelParameters, get_model_type_by_name
from pldepth_amd.models.PLDepthNet import get_pl_depth_net
from pldepth_amd.optimizers import Adam
from pldepth_amd.PLDepth import synthetic_hrwsi

pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("fixed_schedules")]


def test_val_rankings_and_val_loss(cuda):
    B, H, L, R, Rv, seed = 2, 64, 5, 20, 30, 0
    mp = ModelParameters()
    mp.set_parameter("model_type", get_model_type_by_name("ff_effnet"))
    mp.set_parameter("ranking_size", L)
    mp.set_parameter("rankings_per_image", R)
    mp.set_parameter("val_rankings_per_img", Rv)
    mp.set_parameter("batch_size", B)
    mp.set_parameter("loss_type", DepthLossType.NLL)
    mp.set_parameter("seed", seed)
    mp.set_parameter("sampling_strategy", InformationScoreBasedSampling(mp))
    model, pre = get_pl_depth_net(mp, [H, H, 3])
    # lr 1e-5: Adam's first steps move every trainable value by ~lr, and at lr 1e-2 two steps
    # already put this random-init net's inference-mode activations at ~1e7 (see below)
    model.compile(loss=HourglassNegativeLogLikelihood(L, B), optimizer=Adam(1e-5, amsgrad=True))
    imgs, gts, masks = synthetic_hrwsi(9, H, H, seed=3)
    n_val = 5  # 2 full val batches; the ragged fifth image is dropped (drop_remainder)
    prov = HourglassLargeScaleDataProvider(mp, masks[n_val:], masks[:n_val], seed=seed)
    val = prov.provide_val_dataset(pre(imgs[:n_val]), gts[:n_val])
    assert len(val) == 2

    # ---- cached val rankings: Thresholded sampler, Philox draws keyed by the image index
    nc = S.n_candidates(Rv, "thresh")
    for bi, (xb, yb) in enumerate(val):
        y = yb.cpu().numpy()
        assert y.shape == (B, Rv, L, 2)
        i0 = bi * B
        nv = [int((masks[i0 + j] > 0).sum()) for j in range(B)]
        draws = PX.sampler_draws(nv, nc, L, seed + 7919, 0, i0)
        for j in range(B):
            ref, _ = S.sample_masked_point_batch("thresh", masks[i0 + j], gts[i0 + j], Rv, L,
                                                 draws[j].reshape(-1))
            np.testing.assert_array_equal(y[j], ref)
        np.testing.assert_array_equal(xb.cpu().numpy(), pre(imgs[i0:i0 + B]))

    # ---- val_loss, on a one-batch val set. A random-init net in inference mode is only well
    # conditioned on images whose batch statistics its moving statistics hold: on the Keras
    # initial (0, 1), or statistics of other images, the activations grow to ~1e3 by block 6 and
    # ListMLE's exp underflows to log(0) = -inf (as tfr's would). So the moving statistics start
    # from the val batch's own statistics; two training steps then move them by 2 % (momentum
    # 0.99) and the trainable values by ~lr.
    xv = imgs[:B]
    val1 = [(torch.from_numpy(pre(xv)).to(cuda), val[0][1])]
    w = model.get_weights()
    P = {k: torch.tensor(v, dtype=torch.float64) for k, v in w.items()}
    stats = {}
    with torch.no_grad():
        OE.forward(P, torch.tensor(xv, dtype=torch.float64), bn_stats=stats)
    for name, (m, v) in stats.items():
        w[name + "/moving_mean"] = m.numpy().astype(np.float32)
        w[name + "/moving_variance"] = v.numpy().astype(np.float32)
    model.set_weights(w)
    train = prov.provide_train_dataset(pre(imgs[n_val:]), gts[n_val:])
    model.fit(x=train, epochs=1, steps_per_epoch=2, validation_data=val1, verbose=0)
    val_loss = model.history["val_loss"][0]
    assert np.isfinite(val_loss)
    P = {k: torch.tensor(v, dtype=torch.float64) for k, v in model.get_weights().items()}
    # (the moving statistics did move; top_bn's batch mean is ~0: a bias-free 1x1 conv of a
    # training-mode BN output)
    assert not np.allclose(P["top_bn/moving_variance"].numpy(), stats["top_bn"][1].numpy())
    with torch.no_grad():
        pred = OE.forward(P, torch.tensor(xv, dtype=torch.float64), training=False)
    ref, _ = LM.hourglass_nll(val1[0][1].cpu().numpy(), pred.numpy(), B, L)
    assert abs(val_loss - ref) / abs(ref) < 1e-3, (val_loss, ref)
    # evaluate() on the same weights is the same number (Keras evaluate = the val pass)
    assert model.evaluate(val1) == pytest.approx(val_loss, rel=1e-6)
