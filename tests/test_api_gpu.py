"""GPU tests of the reference-shaped API: model factory, loss object, samplers, provider, fit,
predict, save/load — used exactly the way pldepth/PLDepth.py uses its Keras objects."""
import numpy as np
import pytest
import torch

from oracle import listmle as LM
from oracle import sampler as S
from pldepth_amd.data.providers.hourglass_provider import HourglassLargeScaleDataProvider
from pldepth_amd.data.sampling import (InformationScoreBasedSampling,
                                       MaskedRandomSamplingStrategy,
                                       PurelyMaskedRandomSamplingStrategy,
                                       ThresholdedMaskedRandomSamplingStrategy)
from pldepth_amd.losses.losses_meta import DepthLossType
from pldepth_amd.losses.nll_loss import HourglassNegativeLogLikelihood, NegativeLogLikelihoodLoss
from pldepth_amd.models.models_meta import ModelParameters, get_model_type_by_name
from pldepth_amd.models.PLDepthNet import get_pl_depth_net
from pldepth_amd.optimizers import Adam
from pldepth_amd.PLDepth import synthetic_hrwsi
from pldepth_amd.util.training_utils import SGDRScheduler, TerminateOnNaN

pytestmark = pytest.mark.gpu


def _params(B=2, L=5, R=20, model="ff_effnet"):
    mp = ModelParameters()
    mp.set_parameter("model_type", get_model_type_by_name(model))
    mp.set_parameter("ranking_size", L)
    mp.set_parameter("rankings_per_image", R)
    mp.set_parameter("val_rankings_per_img", R)
    mp.set_parameter("batch_size", B)
    mp.set_parameter("loss_type", DepthLossType.NLL)
    mp.set_parameter("seed", 0)
    return mp


@pytest.mark.parametrize("cls,name", [(ThresholdedMaskedRandomSamplingStrategy, "thresh"),
                                      (InformationScoreBasedSampling, "info"),
                                      (PurelyMaskedRandomSamplingStrategy, "pure"),
                                      (MaskedRandomSamplingStrategy, "masked")])
def test_per_image_sampler_consumes_numpy_rng_like_reference(cuda, golden, cls, name):
    """Seeded like the golden capture, the per-image API reproduces the reference output
    (up to tie order)."""
    ci = 1
    h, w, L, R = [int(v) for v in golden[f"c{ci}_shape"]]
    mask = np.unpackbits(golden[f"c{ci}_mask"])[: h * w].reshape(h, w).astype(np.float32)
    gt = golden[f"c{ci}_codes"].astype(np.float32) / np.float32(255)
    strat = cls(_params(L=L))
    np.random.seed(1000 * ci + len(name))
    out = strat.sample_masked_point_batch(np.zeros((h, w, 3), np.float32), mask, gt, R)
    ref = golden[f"c{ci}_{name}_out"]
    assert out.shape == ref.shape
    np.testing.assert_array_equal(S.canonical_lists(out), S.canonical_lists(ref))


def test_loss_objects(cuda):
    rng = np.random.default_rng(0)
    B, H, R, L = 2, 8, 4, 3
    pred = rng.standard_normal((B, H, H, 1)).astype(np.float32)
    idx = rng.integers(0, H * H, (B, R, L))
    lab = rng.permutation(B * R * L).reshape(B, R, L) / (B * R * L)
    y = np.stack([idx, lab], -1).astype(np.float32)
    loss = HourglassNegativeLogLikelihood(ranking_size=L, batch_size=B)(y, pred)
    ref, _ = LM.hourglass_nll(y, pred, B, L)
    assert abs(loss.item() - ref) / ref < 1e-5
    s = rng.standard_normal((7, L)).astype(np.float32)
    lb = rng.permutation(7 * L).reshape(7, L).astype(np.float32)
    l2 = NegativeLogLikelihoodLoss(L)(lb, s)
    n2, _ = LM.listmle_fwd_bwd(s, lb)
    assert abs(l2.item() - n2.mean()) / n2.mean() < 1e-5


def test_fit_predict_save_load(cuda, tmp_path):
    B, H, L, R = 2, 64, 5, 20
    mp = _params(B, L, R)
    mp.set_parameter("sampling_strategy", InformationScoreBasedSampling(mp))
    model, pre = get_pl_depth_net(mp, [H, H, 3])
    imgs, gts, masks = synthetic_hrwsi(8, H, H, seed=0)
    model.compile(loss=HourglassNegativeLogLikelihood(L, B), optimizer=Adam(0.01, amsgrad=True))
    prov = HourglassLargeScaleDataProvider(mp, masks[2:], masks[:2], augmentation=True)
    train = prov.provide_train_dataset(pre(imgs[2:]), gts[2:])
    val = prov.provide_val_dataset(pre(imgs[:2]), gts[:2])
    sched = SGDRScheduler(min_lr=0.04, max_lr=0.01, steps_per_epoch=3, lr_decay=0.9,
                          cycle_length=2, mult_factor=1)
    w0 = model.get_weights()
    model.fit(x=train, epochs=2, steps_per_epoch=3, callbacks=[TerminateOnNaN(), sched],
              validation_data=val, verbose=0)
    w1 = model.get_weights()
    # (val_loss runs BN on moving statistics, which after 6 steps at momentum 0.99 are far from
    # the batch statistics of a random-init net: it may legitimately overflow, as in Keras)
    assert len(model.history["loss"]) == 2 and len(model.history["val_loss"]) == 2
    assert np.isfinite(model.history["loss"]).all()
    assert not np.allclose(w0["dec_conv0/kernel"], w1["dec_conv0/kernel"])  # trained
    np.testing.assert_array_equal(w0["top_conv/kernel"], w1["top_conv/kernel"])  # frozen
    assert not np.allclose(w0["top_bn/gamma"], w1["top_bn/gamma"])  # BN trains
    assert sched.history["lr"][0] == 0.01 and sched.history["lr"][-1] > 0.01  # LR rises
    p1 = model.predict(imgs[:3])
    assert p1.shape == (3, H, H, 1)
    path = str(tmp_path / "w.npz")
    model.save_weights(path)
    model2, _ = get_pl_depth_net(mp, [H, H, 3])
    model2.compile(loss=HourglassNegativeLogLikelihood(L, B), optimizer=Adam(0.01, amsgrad=True))
    model2.load_weights(path)
    np.testing.assert_array_equal(model2.predict(imgs[:3]), p1)
    # Keras HDF5: weights file (load_weights, PLDepth.py:136-137) and whole-model file with the
    # Adam slots (model.save, :181 -> load_model, run_scripts/rnd_on_info_pretrain.py:98)
    h5w = str(tmp_path / "w.h5")
    model.save_weights(h5w)
    model3, _ = get_pl_depth_net(mp, [H, H, 3])
    assert model3.load_weights(h5w) == "name"
    np.testing.assert_array_equal(model3.predict(imgs[:3]), p1)
    h5m = str(tmp_path / "m.h5")
    model.save(h5m)
    from pldepth_amd.models import load_model
    model4 = load_model(h5m)
    model4.compile(loss=HourglassNegativeLogLikelihood(L, B), optimizer=Adam(0.01, amsgrad=True))
    np.testing.assert_array_equal(model4.predict(imgs[:3]), p1)
    for a, b in zip(model.engine.adam_state(), model4.engine.adam_state()):
        assert torch.equal(a, b)
    assert int(model4.trainer.step_dev.item()) == int(model.trainer.step_dev.item())
    # one more identical step on both: resume is exact
    xb, yb = next(iter(train))
    model4.optimizer.lr = model.optimizer.lr
    model.train_on_batch(xb, yb)
    model4.train_on_batch(xb, yb)
    # (equal up to the float-atomic summation order of ListMLE's duplicate-pixel scatter)
    np.testing.assert_allclose(model.get_weights()["dec_conv2/kernel"],
                               model4.get_weights()["dec_conv2/kernel"], rtol=1e-4, atol=1e-6)


def test_redweb_factory_fit_predict(cuda):
    """ff_redweb through the reference's factory: (model, caffe preprocess_fn), compile, fit."""
    B, H, L, R = 2, 64, 5, 20
    mp = _params(B, L, R, model="ff_redweb")
    mp.set_parameter("sampling_strategy", InformationScoreBasedSampling(mp))
    model, pre = get_pl_depth_net(mp, [H, H, 3])
    imgs, gts, masks = synthetic_hrwsi(4, H, H, seed=1)
    x = pre(imgs)
    assert np.allclose(x[..., 0], imgs[..., 2] - 103.939, atol=1e-4)  # BGR, caffe means
    model.compile(loss=HourglassNegativeLogLikelihood(L, B), optimizer=Adam(0.01, amsgrad=True))
    prov = HourglassLargeScaleDataProvider(mp, masks, masks[:2], augmentation=False)
    w0 = model.get_weights()
    model.fit(x=prov.provide_train_dataset(x, gts), epochs=1, steps_per_epoch=2, verbose=0)
    w1 = model.get_weights()
    assert np.isfinite(model.history["loss"]).all()
    assert not np.allclose(w0["ffl0/conv0/kernel"], w1["ffl0/conv0/kernel"])
    np.testing.assert_array_equal(w0["conv3_block2_2_conv/kernel"],
                                  w1["conv3_block2_2_conv/kernel"])  # encoder convs frozen
    assert not np.allclose(w0["conv3_block2_2_bn/gamma"], w1["conv3_block2_2_bn/gamma"])
    assert model.predict(x[:3]).shape == (3, H, H, 1)
