"""Debug: a resumed model (model.save -> load_model) vs the original, one identical step."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from pldepth_amd.data.providers.hourglass_provider import HourglassLargeScaleDataProvider
from pldepth_amd.data.sampling import InformationScoreBasedSampling
from pldepth_amd.losses.nll_loss import HourglassNegativeLogLikelihood
from pldepth_amd.models import load_model
from pldepth_amd.models.PLDepthNet import get_pl_depth_net
from pldepth_amd.optimizers import Adam
from pldepth_amd.PLDepth import synthetic_hrwsi
from tests.test_api_gpu import _params

torch.cuda.set_device(0)
B, H, L, R = 2, 64, 5, 20
mp = _params(B, L, R)
mp.set_parameter("sampling_strategy", InformationScoreBasedSampling(mp))
model, pre = get_pl_depth_net(mp, [H, H, 3])
imgs, gts, masks = synthetic_hrwsi(8, H, H, seed=0)
model.compile(loss=HourglassNegativeLogLikelihood(L, B), optimizer=Adam(0.01, amsgrad=True))
prov = HourglassLargeScaleDataProvider(mp, masks[2:], masks[:2], augmentation=True)
train = prov.provide_train_dataset(pre(imgs[2:]), gts[2:])
model.fit(x=train, epochs=1, steps_per_epoch=3, verbose=0)
model.save("/tmp/m.h5")
m4 = load_model("/tmp/m.h5")
m4.compile(loss=HourglassNegativeLogLikelihood(L, B), optimizer=Adam(0.01, amsgrad=True))
xb, yb = next(iter(train))
m4.optimizer.lr = model.optimizer.lr


def state(m):
    e = m.engine
    return {"params": e.params.buf.clone(), "stats": e.stats.buf.clone(),
            "frozen": e.frozen.buf.clone(), **{k: t.clone() for k, t in
                                              zip(("m", "v", "vh"), e.adam_state())},
            "step": m.trainer.step_dev.clone()}


s1, s4 = state(model), state(m4)
for k in s1:
    print("before", k, bool(torch.equal(s1[k], s4[k])))
l1 = model.train_on_batch(xb, yb)
l4 = m4.train_on_batch(xb, yb)
print("loss", l1, l4)
g1, g4 = model.engine.grads.buf, m4.engine.grads.buf
print("grads rel", float((g1 - g4).abs().max() / g4.abs().max()))
for name in model.engine.params.names()[:6] + ["dec_conv2/kernel", "dec_conv5/bias"]:
    a, b = model.engine.grads[name], m4.engine.grads[name]
    print(name, float((a - b).abs().max()), float(b.abs().max()))
p1, p4 = state(model), state(m4)
for k in p1:
    print("after", k, float((p1[k].double() - p4[k].double()).abs().max()))
# same batch, eager step on the ORIGINAL model's trainer from a re-loaded state
print("pred", float((model.engine.act["pred"] - m4.engine.act["pred"]).abs().max()))
print("x", float((model.trainer.x - m4.trainer.x).abs().max()),
      "y", float((model.trainer.y_true - m4.trainer.y_true).abs().max()))
