"""Parity at the benchmark's own configurations and arithmetic (BASELINE.json configs).

* cfg2 arithmetic: ff_effnet at 448x448 with bf16x3 convs everywhere (what the bench times at
  batch 32) — every trainable gradient against the fp64 oracle, next to the fp32 restatement's
  own error on the same input.
* drop-connect (on in every timed step): HIP keep scales bit-exact vs the Philox restatement
  (oracle/philox.py), keep rate and 1/(1-rate) scale, forward + gradients with those scales
  injected into the oracle (oracle/effnet.py forward(drop_scales=...)).
* cfg1: one whole ReplicaTrainer step (GPU sampler -> fwd -> ListMLE -> bwd -> Adam-AMSGrad) at
  224x224, B=2, L=2, R=100 against the oracle chain (sampler bit-exact, loss, gradients, update).
* cfg3: ff_redweb (ResNet-50 + ReDWeb) at 448x448 against oracle/redweb.py.
* cfg5: the full-size ListMLE (B=32, R=1000, L=64: 2,048,000 list elements, heavy duplicate
  pixels) against oracle/listmle.py.

Gradient bar (BASELINE.json: 1e-3 relative): per tensor 1e-3 wherever the fp32 restatement of
the reference semantics itself lands within 1e-3 of fp64, else 2x the fp32 restatement's own
error; over all tensors together a global rel-L2 within max(1e-3, 2x the fp32 restatement's).
The gradients of the reference semantics are themselves ill-conditioned at the 1e-3 level:
training-mode BN cancels most of each incoming gradient, and
an exact fp32 implementation lands ~1 % (median per tensor) from fp64 at batch 2 AND at the
bench's batch 32 (ff_effnet 5 of 98 tensors within 1e-3, ff_redweb 3 of 237; profiles/r03_parity).
bf16x3 products carry ~2^8 the rounding of fp32 ones; measured HIP / fp32-restatement error
ratios: median 0.90 (ff_effnet) / 1.03 (ff_redweb) at batch 32, worst 2.3. Reports of every tensor
are written to $PLD_REPORT_DIR when set.
Round 4 found where that ill-conditioning comes from for ff_effnet: decoder pre-activations within
rounding of 0 take the other ReLU branch in one implementation (one such pixel passes its whole
gradient or none of it). Measured against the fp64 gradient along each implementation's OWN
decoder ReLU branches (the oracle's relu_masks), every cfg1 tensor of both HIP and the fp32
restatement lands within 1e-3 (HIP global rel-L2 8.6e-5); the ff_effnet tests here use that
flip-aware reference with the strict 1e-3 bar and report the plain comparison and the flip counts
beside it. The ff_redweb tests are flip-aware at all 86 ReLU sites; their per-tensor bar comes from
TWO fp32 restatements (oneDNN and native convolutions): 1e-3 wherever both are within 5e-4, else
SPREAD (2.0) x the worse of the two, with one NAMED exception (FORWARD_ORIGIN) whose excess is
traced to the forward activations and checked by decomposition instead (check_gradients).
Every flip-aware test also checks that each HIP branch flip lies where the fp64 pre-activation is
within rounding of 0 (FLIP_MARGIN), so a wrong forward branch cannot hide in the flip-aware
reference.
"""
import json
import os

import numpy as np
import pytest
import torch

from oracle import effnet as OE
from oracle import listmle as LM
from oracle import philox as PX
from oracle import redweb as OR
from oracle import sampler as S
from oracle.adam import adam_amsgrad_step
from pldepth_amd import kernels as K
from pldepth_amd.models.effnet_ff import EffNetFF

pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("fixed_schedules")]
TOL = 1e-3


def rel(a, b):
    a = torch.as_tensor(a).detach().double().cpu()
    b = torch.as_tensor(b).detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp(min=1e-30))


def make_rankings(rng, B, H, W, R, L):
    idx = rng.integers(0, H * W, (B, R, L))
    lab = rng.permutation(B * R * L).reshape(B, R, L) / (B * R * L)
    lab = -np.sort(-lab, axis=-1)
    return np.ascontiguousarray(np.stack([idx.astype(np.float32), lab.astype(np.float32)], -1))


def report(name, obj):
    d = os.environ.get("PLD_REPORT_DIR")
    if d:
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, f"parity_{name}.json"), "w") as f:
            json.dump(obj, f, indent=1)


def effnet_structural_zero(name, dropped=()):
    """exact-arithmetic zeros (tests/test_model_gpu.py::_structural_zero). A project_bn beta
    stops being one when drop-connect scales its block's residual branch differently per image
    (`dropped`: those block names): the constant then varies across the batch and survives the
    next BN."""
    if name.endswith("project_bn/beta"):
        return name[:-len("project_bn/beta")] not in dropped
    return name.startswith("dec_conv") and name.endswith("/bias")


def _nonuniform(drop):
    return {k for k, v in drop.items() if float(v.max()) != float(v.min())}


# (round 3 kept dec_conv4/kernel as an "ill-conditioned" exception: its plain distance from fp64
# moved between 6.7e-4 and 1.84e-3 with the arithmetic of one upstream layer. Round 4 traced it
# to decoder ReLU branch flips: along HIP's own branches it is 1.4e-5 from fp64 at batch 32, and
# the ff_effnet tests compare flip-aware with no exception.)


def check_gradients(tag, hip, g64, g32, structural_zero, g64_32=None, extra=None, second=None,
                    exceptions=None):
    """The bar of the module docstring; returns the per-tensor report. g64_32: the fp64
    reference the fp32 restatement is measured against (default g64; the flip-aware form gives
    each implementation the fp64 gradient along its own ReLU branches). Per tensor: 1e-3
    wherever the fp32 restatement meets 1e-3, else twice the fp32 restatement's own error.
    second = (g32b, g64_32b): a second fp32 restatement (the same semantics with torch's native
    convolutions instead of oneDNN: another summation order) and its flip-aware fp64 reference.
    With it the per-tensor bar follows how well-conditioned the tensor is by BOTH fp32
    restatements: 1e-3 wherever both are within 1e-3 / 2, else SPREAD (2.0) x the larger of their
    errors (1e-3 floor) — so wherever the two agree (within 1.5x, as they do on all but a few
    tensors) HIP stays within 2x of both. exceptions = {tensor: (ok, note)}: tensors whose bar
    is replaced by a check the caller made (FORWARD_ORIGIN); reported with both."""
    g64_32 = g64 if g64_32 is None else g64_32
    exceptions = exceptions or {}
    keys = [k for k in g64 if not structural_zero(k)]
    rows, fails = {}, []
    for k in keys:
        e_hip, e32 = rel(hip[k], g64[k]), rel(g32[k], g64_32[k])
        if second is None:
            bar = TOL if e32 <= TOL else 2.0 * e32
            rows[k] = {"hip": e_hip, "fp32_restatement": e32, "bar": bar}
        else:
            e32b = rel(second[0][k], second[1][k])
            worst = max(e32, e32b)
            bar = TOL if worst <= TOL / 2 else max(TOL, SPREAD * worst)
            rows[k] = {"hip": e_hip, "fp32_restatement": e32, "fp32_restatement_native_conv": e32b,
                       "bar": bar}
        if k in exceptions:
            ok, note = exceptions[k]
            rows[k]["exception"] = note
            if not ok:
                fails.append((k, e_hip, note))
        elif e_hip > rows[k]["bar"]:
            fails.append((k, e_hip, e32))
    flat = lambda g: torch.cat([torch.as_tensor(g[k]).detach().double().cpu().flatten()
                                for k in keys])
    a, b, c, b32 = flat(hip), flat(g64), flat(g32), flat(g64_32)
    glob = {"hip_rel_l2": float((a - b).norm() / b.norm()),
            "fp32_rel_l2": float((c - b32).norm() / b32.norm()),
            "cos": float(a @ b / (a.norm() * b.norm())),
            "tensors": len(keys),
            "tensors_fp32_within_1e-3": sum(r["fp32_restatement"] <= TOL for r in rows.values()),
            "tensors_hip_within_1e-3": sum(r["hip"] <= TOL for r in rows.values()),
            "tensors_strict_bar": sum(r["bar"] <= TOL for r in rows.values()),
            "exceptions": sorted(exceptions)}
    if second is not None:
        d, e = flat(second[0]), flat(second[1])
        glob["fp32_native_conv_rel_l2"] = float((d - e).norm() / e.norm())
    scale = float(b.abs().max())
    for k in g64:
        if structural_zero(k):
            assert float(torch.as_tensor(hip[k]).abs().max()) <= 1e-3 * scale + 1e-6, k
    report(tag, dict({"global": glob, "tensors": rows}, **(extra or {})))
    print(f"[{tag}] {glob}")
    assert not fails, fails[:10]
    assert glob["hip_rel_l2"] <= max(TOL, 2.0 * glob["fp32_rel_l2"],
                                     2.0 * glob.get("fp32_native_conv_rel_l2", 0.0))
    return glob


# A BN-gamma gradient is sum(dz * xhat) over the batch: where that sum cancels, the error of the
# FORWARD activations xhat is amplified into it, and the pattern of that error (set by the chaotic
# ResNet-50 encoder under training-mode BN: fp32 rounding of conv2-stage inputs grows ~100x by
# conv5) decides how much. tools/exp_redweb_dz.py (round 6,
# profiles/r06_redweb_dz.txt) traced the one ff_redweb tensor over 2x both fp32 restatements in
# test_cfg3_redweb_448 (ffl2/block_down/bn3/gamma: HIP 1.52e-3, oneDNN 6.78e-4, native 6.71e-4,
# ratio 2.24): with every decoder conv exact fp32, forward and backward, it moves < 1 %; fed the
# same dL/dpred along the same ReLU branches, every HIP activation gradient of the decoder is
# within 3.3e-5 of fp64, and the gamma gradient rebuilt from HIP's dz with fp64's xhat is 5.5e-4
# from fp64 while HIP's dz with HIP's own xhat gives 1.85e-3 — the excess enters through xhat.
# For these named BNs the test therefore checks the two halves instead of the sum: the gradient
# from HIP's dz and fp64's xhat within the tensor's normal bar (HIP's backward arithmetic), and
# HIP's forward xhat within 2x the fp32 restatement's own xhat error (HIP's forward arithmetic).
FORWARD_ORIGIN = {"cfg3_redweb448_mixed": ("ffl2/block_down/bn3",)}


def _bn_capture(store, names):
    """An oracle/redweb.py _bn wrapper recording the pre-BN input of the named BNs."""
    orig = OR._bn

    def bn(P_, name, xx, eps):
        if name in names:
            store[name] = xx.detach()
        return orig(P_, name, xx, eps)
    return orig, bn


def _xhat(xx, eps):
    mu = xx.mean(dim=(0, 2, 3), keepdim=True)
    var = ((xx - mu) ** 2).mean(dim=(0, 2, 3), keepdim=True)
    return (xx - mu) / torch.sqrt(var + eps)


def tensor_bar(k, g32, g64_32, second):
    """check_gradients' per-tensor bar (with `second`) for tensor k."""
    worst = max(rel(g32[k], g64_32[k]), rel(second[0][k], second[1][k]))
    return TOL if worst <= TOL / 2 else max(TOL, SPREAD * worst)


def forward_origin_checks(tag, eng, bn_in64, bn_in32, g64h, relu_masks, bars):
    """{gamma tensor: (ok, note)} for FORWARD_ORIGIN[tag] (see there). bars: tensor -> its normal
    per-tensor bar (check_gradients' rule)."""
    out = {}
    for name in FORWARD_ORIGIN.get(tag, ()):
        bt, i = name.rsplit("/bn", 1)
        i = int(i)
        d = next(f for f in eng.ffls if bt.startswith(f["name"] + "/"))
        bn = d["left" if "block_left" in bt else "down"]["bns"][i]
        pre, site = f"{bt}/pre{i}", f"{bt}/act{i}"
        xh_h = ((eng.act[pre].double() - bn.mean.double()) * bn.invstd.double()) \
            .permute(0, 3, 1, 2).cpu()
        xh_64 = _xhat(bn_in64[name].double(), OR.DEC_BN_EPS)
        xh_32 = _xhat(bn_in32[name].double(), OR.DEC_BN_EPS)
        dz_h = eng.gact[site].permute(0, 3, 1, 2).double().cpu() * relu_masks[site].double()
        k = name + "/gamma"
        e_bwd = rel((dz_h * xh_64).sum(dim=(0, 2, 3)), g64h[k])
        e_xh, e_xh32 = rel(xh_h, xh_64), rel(xh_32, xh_64)
        ok = e_bwd <= bars[k] and e_xh <= 2.0 * e_xh32
        out[k] = (ok, {"gamma_from_hip_dz_fp64_xhat": e_bwd, "bar": bars[k],
                       "hip_xhat": e_xh, "fp32_xhat": e_xh32})
    return out


def native_conv_restatement(O, P32, x32, dref32, P, x64, dref64, **kw):
    """The second fp32 restatement (check_gradients' `second`): the oracle with torch's native
    convolutions (oneDNN off), its own ReLU branches, and the fp64 gradient along them."""
    b = {}
    with torch.backends.mkldnn.flags(enabled=False):
        with torch.no_grad():
            O.forward(P32, x32, relu_branches=b, **kw)
        g32b = O.train_step_grads(P32, x32, dref32, **kw)[0]
    g64b = O.train_step_grads(P, x64, dref64, relu_masks=b, **kw)[0]
    return g32b, g64b


# ------------------------------------------------------------ cfg2 arithmetic at 448x448
def test_effnet_448_bf16x3_gradients(cuda, fixed_schedules):
    B, H, R, L = 2, 448, 100, 5
    eng = EffNetFF((H, H, 3), B, seed=0, conv_math="bf16x3")
    eng.drop_connect = False
    rng = np.random.default_rng(5)
    x = rng.random((B, H, H, 3)).astype(np.float32)
    weights = eng.get_weights()
    eng.act["input"].copy_(torch.from_numpy(x))
    pred = eng.forward(training=True)
    y = make_rankings(rng, B, H, H, R, L)
    loss, dpred, _ = K.listmle_fwd_bwd(pred, torch.from_numpy(y).to(cuda), B, R, L)
    eng.backward(dpred)
    torch.cuda.synchronize()
    P = {k: torch.tensor(v, dtype=torch.float64) for k, v in weights.items()}
    x64 = torch.tensor(x, dtype=torch.float64)
    with torch.no_grad():
        pred_ref = OE.forward(P, x64)
    loss_ref, dpred_ref = LM.hourglass_nll(y, pred_ref.numpy(), B, L)
    assert rel(pred, pred_ref) < TOL
    assert abs(loss.item() - loss_ref) / abs(loss_ref) < TOL
    glob = effnet_grads_flip_aware("effnet448_bf16x3", eng, weights, x, dpred_ref,
                                   effnet_structural_zero)
    assert glob["cos"] > 0.9999


# ------------------------------------------------------------------- drop-connect
def hip_decoder_relu_masks(eng, weights):
    """The decoder ReLU branches the HIP forward took, as [N, C, H, W] masks for
    OE.forward(relu_masks=...). The kernels (the BN prologue of upsample2x_fwd_cell and the BN
    backward, csrc/resample.hip / bn.hip) decide z = fma((x - mean) * invstd, gamma, beta) > 0 in
    fp32 with the step's batch statistics and the pre-update gamma / beta: the
    product (x - mean) * invstd is formed in fp32 as they do, and the sign of the fused
    multiply-add is the sign of its exact value, which fp64 gives exactly (the fp32 x fp32
    product is exact in fp64 and a rounded sum keeps the exact sum's sign)."""
    out = {}
    for i, (conv, bn, skip) in enumerate(eng.dec):
        pre = eng.act[f"dec{i}_pre"].float().cpu()
        xh = (pre - bn.mean.float().cpu()) * bn.invstd.float().cpu()
        ga = torch.tensor(weights[f"dec_bn{i}/gamma"], dtype=torch.float32).double()
        be = torch.tensor(weights[f"dec_bn{i}/beta"], dtype=torch.float32).double()
        z = xh.double() * ga + be
        out[i] = (z > 0).permute(0, 3, 1, 2).double()
    return out


# A HIP ReLU branch that differs from fp64's must sit where the fp64 pre-activation is within
# rounding of 0: |z64| at every flipped position <= FLIP_MARGIN x max |z64| of that
# site. The forward activations themselves agree with fp64 to ~1e-4 of their scale (taps,
# test_batch32_bench_policy), so a flip further out means the forward took a wrong branch, which
# the flip-aware gradient comparison would otherwise absorb.
FLIP_MARGIN = 2e-3  # observed (round 5): <= 3e-5 ff_effnet, 4.1e-4 ff_redweb at batch 2

# Per-tensor factor over the worse fp32 restatement where a tensor is not clearly
# well-conditioned (check_gradients' `second`). Round 5 set 2.5 after the one tensor at 2.24
# (a bar fitted to the output); round 6 restores 2.0 and handles that tensor by name
# with the decomposition check of FORWARD_ORIGIN.
SPREAD = 2.0


def flip_margin(z64, hip_mask):
    """max |z64| over the positions where HIP's branch (hip_mask, same layout) differs from
    fp64's, relative to max |z64| (0 when there is no flip)."""
    d = (z64 > 0) != (hip_mask > 0)
    if not bool(d.any()):
        return 0.0
    return float(z64.abs()[d].max() / z64.abs().max())


class FlipProbe(dict):
    """relu_branches for oracle/redweb.py that also measures, per site, flip_margin of the HIP
    branches `hip` against this (fp64) run's pre-activations; stores this run's branches like a
    plain dict."""

    def __init__(self, hip):
        super().__init__()
        self.hip, self.margin = hip, {}

    def record(self, site, x):
        self[site] = x > 0
        if site in self.hip:
            self.margin[site] = flip_margin(x, self.hip[site].to(x.device))


def assert_flip_margins(margins):
    worst = max(margins.items(), key=lambda kv: kv[1]) if margins else (None, 0.0)
    assert worst[1] <= FLIP_MARGIN, ("HIP ReLU branch flipped away from 0", worst)
    return {"worst_site": worst[0], "worst": worst[1], "bar": FLIP_MARGIN}


def effnet_grads_flip_aware(tag, eng, weights, x, dpred_ref, structural_zero, drop=None):
    """check_gradients for an ff_effnet step against the flip-aware reference: HIP vs the fp64
    gradient along HIP's decoder ReLU branches, the fp32 restatement vs fp64 along its own, the
    strict 1e-3 bar; the plain comparison and the per-stage ReLU flip counts go to the report."""
    mh = hip_decoder_relu_masks(eng, weights)
    hip = {k: eng.grads[k] for k in OE.trainable_names(weights)}
    P = {k: torch.tensor(v, dtype=torch.float64) for k, v in weights.items()}
    P32 = {k: torch.tensor(v, dtype=torch.float32) for k, v in weights.items()}
    x64, x32 = torch.tensor(x, dtype=torch.float64), torch.tensor(x)
    d64 = torch.tensor(dpred_ref, dtype=torch.float64)
    drop32 = None if drop is None else {k: v.float() for k, v in drop.items()}
    taps64, taps32 = {}, {}
    with torch.no_grad():
        OE.forward(P, x64, drop_scales=drop, taps=taps64)
        OE.forward(P32, x32, drop_scales=drop32, taps=taps32)
    m32 = {i: (taps32[f"dec{i}_z"] > 0).double() for i in mh}
    flips = {f"dec{i}": {"hip": int(((mh[i] > 0) != (taps64[f"dec{i}_z"] > 0)).sum()),
                         "fp32": int(((m32[i] > 0) != (taps64[f"dec{i}_z"] > 0)).sum())}
             for i in mh}
    margins = {f"dec{i}": flip_margin(taps64[f"dec{i}_z"], mh[i]) for i in mh}
    margin = assert_flip_margins(margins)
    del taps64, taps32
    g64, _ = OE.train_step_grads(P, x64, d64, drop_scales=drop)
    g32, _ = OE.train_step_grads(P32, x32, d64.float(), drop_scales=drop32)
    plain = {k: {"hip": rel(hip[k], g64[k]), "fp32_restatement": rel(g32[k], g64[k])}
             for k in g64}
    del g64
    g64h, _ = OE.train_step_grads(P, x64, d64, drop_scales=drop, relu_masks=mh)
    g64f, _ = OE.train_step_grads(P, x64, d64, drop_scales=drop, relu_masks=m32)
    return check_gradients(tag, hip, g64h, g32, structural_zero, g64_32=g64f,
                           extra={"relu_flips_vs_fp64": flips, "flip_margin": margins,
                                  "flip_margin_check": margin, "plain_comparison": plain})


def _residual_drop_blocks(eng):
    return [(li, blk) for li, blk in enumerate(eng.blocks) if blk["residual"] and blk["rate"] > 0]


@pytest.mark.parametrize("rate", [0.0125, 0.1875, 0.5])
def test_dropconnect_scales_bit_exact_and_keep_rate(cuda, rate):
    n, seed = 8192, 11
    out = torch.empty(n, device=cuda)
    zeros = 0
    for step in range(1, 9):
        K.dropconnect_scales(out, rate, seed, step, layer=7, image_offset=3)
        got = out.cpu().numpy()
        ref = PX.dropconnect_scales(n, rate, seed, step, layer=7, image_offset=3)
        np.testing.assert_array_equal(got, ref)
        zeros += int((got == 0).sum())
        # graph-replayable form (device step counter) is the same stream
        K.dropconnect_scales(out, rate, seed, torch.tensor([step], dtype=torch.int64,
                                                           device=cuda), layer=7, image_offset=3)
        np.testing.assert_array_equal(out.cpu().numpy(), ref)
    keep = got[got != 0]
    assert np.all(keep == np.float32(1) / (np.float32(1) - np.float32(rate)))
    N = 8 * n
    assert abs(zeros / N - rate) < 5 * np.sqrt(rate * (1 - rate) / N)


def test_dropconnect_scales_multi_layer_launch(cuda):
    """Every block's keep factors in one launch (the forward's form): row s is layer
    layers[s]'s stream, host step and device step alike."""
    n, seed, rates, layers = 37, 5, [0.0125, 0.05, 0.1875, 0.5], [1, 4, 9, 15]
    out = torch.empty(len(layers), n, device=cuda)
    for step in (1, (1 << 33) + 3):
        for st in (step, torch.tensor([step], dtype=torch.int64, device=cuda)):
            out.fill_(-1.0)
            K.dropconnect_scales_multi(out, rates, layers, seed, st, image_offset=6)
            got = out.cpu().numpy()
            for s, (r, li) in enumerate(zip(rates, layers)):
                np.testing.assert_array_equal(
                    got[s], PX.dropconnect_scales(n, r, seed, step, layer=li, image_offset=6))


def test_dropconnect_scales_multi_more_layers_than_one_launch(cuda):
    """More blocks than one launch's parameter block (kernels.DC_MAX_LAYERS): split into
    launches, every row still its own layer's stream."""
    n, seed, step = 11, 9, 4
    nl = K.DC_MAX_LAYERS + 5
    rates = [0.01 * (1 + i % 20) for i in range(nl)]
    layers = list(range(2, 2 + nl))
    out = torch.full((nl, n), -1.0, device=cuda)
    K.dropconnect_scales_multi(out, rates, layers, seed, step)
    got = out.cpu().numpy()
    for s, (r, li) in enumerate(zip(rates, layers)):
        np.testing.assert_array_equal(got[s], PX.dropconnect_scales(n, r, seed, step, layer=li))


def test_sampler_draws_bit_exact_vs_philox(cuda):
    nv = np.array([1, 7, 1000, 200704], np.int32)
    d = torch.empty(4, 500, 5, dtype=torch.int32, device=cuda)
    K.sampler_draw(torch.from_numpy(nv).to(cuda), 500, 5, seed=1234, step=(1 << 33) + 7,
                   image_offset=5, draws=d)
    np.testing.assert_array_equal(d.cpu().numpy(),
                                  PX.sampler_draws(nv, 500, 5, 1234, (1 << 33) + 7, 5))


def test_dropconnect_forward_and_gradients(cuda, fixed_schedules):
    """Drop-connect as the timed step runs it: the per-block (step, image)-keyed scales read
    back from the engine and injected into the oracle."""
    B, H, R, L, seed = 4, 128, 24, 5, 0
    eng = EffNetFF((H, H, 3), B, seed=seed, conv_math="fp32")
    eng.drop_connect = True
    blocks = _residual_drop_blocks(eng)
    # a step whose masks drop at least one residual branch (the 1/(1-rate) scale alone is
    # exercised by every kept one)
    step = next(s for s in range(1, 200) if any(
        (PX.dropconnect_scales(B, blk["rate"], seed, s, li) == 0).any() for li, blk in blocks))
    rng = np.random.default_rng(2)
    x = rng.random((B, H, H, 3)).astype(np.float32)
    weights = eng.get_weights()
    eng.act["input"].copy_(torch.from_numpy(x))
    pred = eng.forward(training=True, step=step)
    y = make_rankings(rng, B, H, H, R, L)
    loss, dpred, _ = K.listmle_fwd_bwd(pred, torch.from_numpy(y).to(cuda), B, R, L)
    eng.backward(dpred)
    torch.cuda.synchronize()
    drop = {}
    for li, blk in blocks:
        got = blk["drop"].cpu().numpy()
        np.testing.assert_array_equal(got, PX.dropconnect_scales(B, blk["rate"], seed, step, li))
        drop[blk["name"]] = torch.tensor(got, dtype=torch.float64)
    P = {k: torch.tensor(v, dtype=torch.float64) for k, v in weights.items()}
    x64 = torch.tensor(x, dtype=torch.float64)
    taps = {}
    with torch.no_grad():
        pred_ref = OE.forward(P, x64, drop_scales=drop, taps=taps)
        pred_nodrop = OE.forward(P, x64)
    assert rel(pred_ref, pred_nodrop) > 1e-2  # the masks matter for this input
    for name in ["block2b_output", "block5c_output", "block6d_output", "top_activation"]:
        assert rel(eng.act[name], taps[name].permute(0, 2, 3, 1)) < TOL, name
    assert rel(pred, pred_ref) < TOL
    loss_ref, dpred_ref = LM.hourglass_nll(y, pred_ref.numpy(), B, L)
    assert abs(loss.item() - loss_ref) / abs(loss_ref) < TOL
    nu = _nonuniform(drop)
    assert nu  # at least one block's branch is scaled differently across the batch
    effnet_grads_flip_aware("dropconnect128", eng, weights, x, dpred_ref,
                            lambda k: effnet_structural_zero(k, nu), drop=drop)


# ------------------------------------------------------------------- cfg1: whole step
def test_cfg1_trainer_step_224(cuda, fixed_schedules):
    """BASELINE cfg1 (ff_effnet 224x224, B=2, L=2, R=100, Info sampler): one eager
    ReplicaTrainer step — GPU sampler, forward with drop-connect, ListMLE, backward, Adam —
    against the oracle chain fed the same Philox draws and drop scales."""
    from pldepth_amd.trainer import ReplicaTrainer
    B, H, L, R, lr = 2, 224, 2, 100, 0.01
    tr = ReplicaTrainer((H, H, 3), B, L, R, 1, seed=0)
    eng = tr.engine
    rng = np.random.default_rng(9)
    x = rng.random((B, H, H, 3)).astype(np.float32)
    yy, xx = np.meshgrid(np.linspace(0, 1, H), np.linspace(0, 1, H), indexing="ij")
    gt = np.stack([np.round(255 * (0.5 + 0.3 * np.sin((3 + b) * yy) * np.cos(2 * xx))) / 255
                   for b in range(B)]).astype(np.float32)
    mask = (rng.random((B, H, H)) < 0.9).astype(np.float32)
    weights = eng.get_weights()
    params0 = eng.params.buf.clone()
    tr.set_batch(torch.from_numpy(x).to(cuda), torch.from_numpy(gt).to(cuda),
                 torch.from_numpy(mask).to(cuda))
    tr.step_eager(lr)
    tr.synchronize()
    # sampler: the step's Philox draws, then the reference's gather/sort/score/select, bit-exact
    draws = tr.draws.cpu().numpy()
    nv = [int((mask[b] > 0).sum()) for b in range(B)]
    np.testing.assert_array_equal(draws, PX.sampler_draws(nv, draws.shape[1], L, 0, 1, 0))
    y = tr.y_true.cpu().numpy()
    for b in range(B):
        ref, _ = S.sample_masked_point_batch("info", mask[b], gt[b], R, L, draws[b].reshape(-1))
        np.testing.assert_array_equal(y[b], ref)
    drop = {blk["name"]: torch.tensor(blk["drop"].cpu().numpy(), dtype=torch.float64)
            for li, blk in _residual_drop_blocks(eng)}
    for li, blk in _residual_drop_blocks(eng):
        np.testing.assert_array_equal(drop[blk["name"]].numpy().astype(np.float32),
                                      PX.dropconnect_scales(B, blk["rate"], 0, 1, li))
    P = {k: torch.tensor(v, dtype=torch.float64) for k, v in weights.items()}
    x64 = torch.tensor(x, dtype=torch.float64)
    with torch.no_grad():
        pred_ref = OE.forward(P, x64, drop_scales=drop)
    loss_ref, dpred_ref = LM.hourglass_nll(y, pred_ref.numpy(), B, L)
    assert abs(tr.loss_value() - loss_ref) / abs(loss_ref) < TOL
    # Flip-aware reference: at 224^2 batch 2 a few decoder pre-activations lie within rounding
    # of 0 (dec3: 21 of 200704 within 1e-5 of the largest), and a pixel whose ReLU branch differs
    # passes its whole gradient in one realization and none in the other. One such pixel in a
    # channel whose beta gradient cancels to a small sum sets that tensor's max error
    # (tools/exp_relu_flips.py: the worst dec_bn{i}/beta channel holds a flipped pixel at every
    # stage; the fp32 restatement flips 3-33 pixels per stage, HIP 1-13).
    nu = _nonuniform(drop)
    effnet_grads_flip_aware("cfg1_224", eng, weights, x, dpred_ref,
                            lambda k: effnet_structural_zero(k, nu), drop=drop)
    # Adam-AMSGrad (step 1) applied by the oracle to the step's own gradients
    z = np.zeros(params0.numel(), np.float32)
    p_ref, *_ = adam_amsgrad_step(params0.cpu().numpy(), eng.grads.buf.cpu().numpy(), z, z, z,
                                  lr, 1)
    np.testing.assert_allclose(eng.params.buf.cpu().numpy(), p_ref, rtol=1e-6, atol=1e-7)
    assert int(tr.step_dev.item()) == 2


# ------------------------------------------------------------------- cfg3: ff_redweb 448
def test_cfg3_redweb_448(cuda, fixed_schedules):
    """Whole training step at batch 2 with the encoder in exact fp32 and the decoder bf16x3
    ('mixed'). With bf16x3 in the early encoder too, conv5_block3_out lands 1.2e-3 from fp64 at
    this batch: the conv4/conv5 BNs normalise over 28*28*2 / 14*14*2 values per channel and
    amplify the rounding. The bench's batch-32 arithmetic is checked at batch 32 below."""
    from pldepth_amd.models.redweb_ff import RedWebFF, preprocess_input
    B, H, R, L = 2, 448, 100, 5
    eng = RedWebFF((H, H, 3), B, seed=0, conv_math="mixed")
    rng = np.random.default_rng(4)
    x = preprocess_input(rng.random((B, H, H, 3)).astype(np.float32))
    weights = eng.get_weights()
    eng.act["input"].copy_(torch.from_numpy(x))
    pred = eng.forward(training=True)
    # the ReLU branches the HIP forward took (materialised outputs, read before the backward)
    mr = {st: (eng.act[st] > 0).permute(0, 3, 1, 2).cpu() for st in OR.relu_sites()}
    y = make_rankings(rng, B, H, H, R, L)
    loss, dpred, _ = K.listmle_fwd_bwd(pred, torch.from_numpy(y).to(cuda), B, R, L)
    eng.backward(dpred)
    torch.cuda.synchronize()
    P = {k: torch.tensor(v, dtype=torch.float64) for k, v in weights.items()}
    x64 = torch.tensor(x, dtype=torch.float64)
    taps, taps32 = {}, {}
    P32 = {k: torch.tensor(v, dtype=torch.float32) for k, v in weights.items()}
    b64, b32 = FlipProbe(mr), {}
    tag = "cfg3_redweb448_mixed"
    bn_in64, bn_in32 = {}, {}
    named = FORWARD_ORIGIN.get(tag, ())
    orig, cap64 = _bn_capture(bn_in64, named)
    _, cap32 = _bn_capture(bn_in32, named)
    try:
        with torch.no_grad():
            OR._bn = cap64
            pred_ref = OR.forward(P, x64, taps=taps, preprocessed=True, relu_branches=b64)
            OR._bn = cap32
            OR.forward(P32, torch.tensor(x), taps=taps32, preprocessed=True, relu_branches=b32)
    finally:
        OR._bn = orig
    for name in ["conv1_relu", "conv2_block3_out", "conv3_block4_out", "conv4_block3_out",
                 "conv5_block3_out", "ffl0", "ffl1"]:
        mine = eng.act[name if not name.startswith("ffl") else name + "/out"]
        ref = taps[name].permute(0, 2, 3, 1)
        # 53 training-mode BNs deep, the fp32 restatement itself reaches ~1e-3 at conv5
        bar = max(TOL, 2.0 * rel(taps32[name].permute(0, 2, 3, 1), ref))
        assert rel(mine, ref) < bar, (name, rel(mine, ref), bar)
    assert rel(pred, pred_ref) < TOL
    loss_ref, dpred_ref = LM.hourglass_nll(y, pred_ref.numpy(), B, L)
    assert abs(loss.item() - loss_ref) / abs(loss_ref) < TOL
    assert rel(dpred, torch.tensor(dpred_ref)) < TOL
    # flip-aware at every ReLU site: HIP against the fp64 gradient along
    # HIP's branches, the fp32 restatement along its own, the strict bar
    margin = assert_flip_margins(dict(b64.margin))
    flips = {"hip": sum(int((mr[st] != b64[st]).sum()) for st in OR.relu_sites()),
             "fp32": sum(int((b32[st] != b64[st]).sum()) for st in OR.relu_sites())}
    dref = torch.tensor(dpred_ref, dtype=torch.float64)
    g64h, _ = OR.train_step_grads(P, x64, dref, preprocessed=True, relu_masks=mr)
    g64f, _ = OR.train_step_grads(P, x64, dref, preprocessed=True, relu_masks=b32)
    g32, _ = OR.train_step_grads(P32, torch.tensor(x), dref.float(), preprocessed=True)
    second = native_conv_restatement(OR, P32, torch.tensor(x), dref.float(), P, x64, dref,
                                     preprocessed=True)
    zeros = {"aol/conv0/bias", "aol/conv1/bias", "aol/conv2/bias"}
    bars = {n + "/gamma": tensor_bar(n + "/gamma", g32, g64f, second) for n in named}
    exc = forward_origin_checks(tag, eng, bn_in64, bn_in32, g64h, mr, bars)
    check_gradients(tag, {k: eng.grads[k] for k in g64h}, g64h, g32,
                    lambda k: k in zeros, g64_32=g64f,
                    extra={"relu_flips_vs_fp64_total": flips, "flip_margin": dict(b64.margin),
                           "flip_margin_check": margin}, second=second, exceptions=exc)


# ------------------------------------------------------------------- cfg5: full ListMLE
def test_cfg5_listmle_full_size(cuda):
    """B=32, 448x448, R=1000, L=64: E = 2,048,000 gathered scores. Indices come from a pool of
    20,000 pixels per image, so every pixel is hit ~100 times (duplicate-pixel scatter-add) and
    lists hold repeated pixels as the sampler's with-replacement draws do."""
    B, H, R, L = 32, 448, 1000, 64
    rng = np.random.default_rng(64)
    pred = (0.5 * rng.standard_normal((B, H, H, 1))).astype(np.float32)
    pool = np.stack([rng.choice(H * H, 20000, replace=False) for _ in range(B)])
    idx = np.take_along_axis(pool, rng.integers(0, 20000, (B, R * L)), 1).reshape(B, R, L)
    lab = rng.random((B, R, L)).astype(np.float32)
    lab = -np.sort(-lab, axis=-1)
    y = np.ascontiguousarray(np.stack([idx.astype(np.float32), lab], -1))
    loss_ref, dpred_ref = LM.hourglass_nll(y, pred, B, L)
    loss, dpred, nll = K.listmle_fwd_bwd(torch.from_numpy(pred).to(cuda),
                                         torch.from_numpy(y).to(cuda), B, R, L)
    torch.cuda.synchronize()
    assert abs(loss.item() - loss_ref) / abs(loss_ref) < 1e-5
    assert rel(dpred, torch.from_numpy(dpred_ref)) < 1e-5
    hit = np.zeros(B * H * H, bool)
    hit[(idx + (np.arange(B) * H * H)[:, None, None]).reshape(-1)] = True
    d = dpred.cpu().numpy().reshape(-1)
    assert np.all(d[~hit] == 0)  # untouched pixels get exactly zero gradient


# ------------------------------------------------------------------- empty masks
def test_sampler_empty_mask_is_defined(cuda):
    """an all-zero mask compacts nothing; the GPU path emits a defined all-invalid
    list (index 0, label -1, masked by ListMLE) instead of reading unwritten memory, and the
    per-image reference entry raises like np.random.randint(0) does (sampling.py:113)."""
    from pldepth_amd.data.sampling import InformationScoreBasedSampling
    from pldepth_amd.models.models_meta import ModelParameters
    mp = ModelParameters()
    mp.set_parameter("ranking_size", 5)
    st = InformationScoreBasedSampling(mp)
    H = 32
    gt = torch.rand(2, H, H, device=cuda)
    mask = torch.ones(2, H, H, device=cuda)
    mask[1] = 0
    out = st.sample_batch_gpu(gt, mask, 10, seed=1, step=1).cpu().numpy()
    assert np.all(out[1, :, :, 0] == 0) and np.all(out[1, :, :, 1] == -1)
    assert np.all(out[0, :, :, 1] >= 0)
    with pytest.raises(ValueError):
        st.sample_masked_point_batch(None, np.zeros((H, H)), np.ones((H, H)), 10)


# ------------------------------------------------- the bench's arithmetic at its own batch
def _oracle_step(O, P, x, y, B, L, taps=None, **kw):
    """One oracle forward (taps recorded) + hourglass ListMLE + backward: (pred, loss, dpred,
    grads of the trainable tensors). dpred is taken from this forward's own prediction."""
    names = set(O.trainable_names(P))
    Q = {k: (v.detach().clone().requires_grad_(True) if k in names else v.detach())
         for k, v in P.items()}
    out = O.forward(Q, x, taps=taps, **kw)
    loss, dpred = LM.hourglass_nll(y, out.detach().double().numpy(), B, L)
    out.backward(torch.tensor(dpred, dtype=out.dtype))
    if taps is not None:
        for k in list(taps):
            taps[k] = taps[k].detach()
    grads = {k: Q[k].grad.detach() for k in names}
    return out.detach(), loss, dpred, grads


@pytest.mark.timeout(1500)
@pytest.mark.parametrize("model", ["ff_effnet", "ff_redweb"])
def test_batch32_bench_policy(cuda, model, bench_schedules):
    """cfg2 / cfg3 exactly as the bench runs them: 448x448, batch 32, the default 'auto' conv
    policy (ff_effnet: bf16x3 everywhere; ff_redweb: bf16x3 except the stem and conv2 stage,
    RedWebFF.exact_stages) and the bench's own persisted conv schedule table
    (kernels.DEFAULT_SCHEDULES, the bench_schedules fixture). Forward taps, prediction, loss
    and every trainable gradient against the fp64 oracle, next to the torch-CPU fp32 restatement of the same reference semantics on
    the same input: every tap and the prediction within max(1e-3, 2x the fp32 restatement's
    error), the loss within 1e-3, the gradients by check_gradients' bar (1e-3 wherever the
    fp32 restatement meets it). Reports go to $PLD_REPORT_DIR."""
    B, H, R, L = 32, 448, 100, 5
    rng = np.random.default_rng(32)
    x = rng.random((B, H, H, 3)).astype(np.float32)
    if model == "ff_effnet":
        eng = EffNetFF((H, H, 3), B, seed=0, conv_math="auto")
        eng.drop_connect = False
        O, kw = OE, {}
        names = ["stem_activation", "block2a_output", "block3a_expand_activation",
                 "block5c_output", "block7a_output", "top_activation"]
        mine = eng.tap
        zero = effnet_structural_zero
    else:
        from pldepth_amd.models.redweb_ff import RedWebFF, preprocess_input
        eng = RedWebFF((H, H, 3), B, seed=0, conv_math="auto")
        x = preprocess_input(x)
        O, kw = OR, {"preprocessed": True}
        names = ["conv1_relu", "conv2_block3_out", "conv3_block4_out", "conv4_block3_out",
                 "conv5_block3_out", "ffl0", "ffl1", "ffl2"]
        mine = lambda n: eng.act[n if not n.startswith("ffl") else n + "/out"]
        zeros = {"aol/conv0/bias", "aol/conv1/bias", "aol/conv2/bias"}
        zero = lambda k: k in zeros
    assert eng.enc_math == "auto"
    weights = eng.get_weights()
    eng.act["input"].copy_(torch.from_numpy(x))
    pred = eng.forward(training=True)
    # ff_redweb: every ReLU branch the HIP forward took (its materialised ReLU outputs, read
    # before the backward reuses any buffer), for the flip-aware gradient reference
    mr = ({st: (eng.act[st] > 0).permute(0, 3, 1, 2).cpu() for st in OR.relu_sites()}
          if model == "ff_redweb" else None)
    y = make_rankings(rng, B, H, H, R, L)
    loss, dpred, _ = K.listmle_fwd_bwd(pred, torch.from_numpy(y).to(cuda), B, R, L)
    eng.backward(dpred)
    torch.cuda.synchronize()
    hip_taps = {n: mine(n).detach().cpu().double() for n in names}
    hip_pred, hip_loss = pred.detach().cpu().double(), loss.item()
    hip_grads = {k: eng.grads[k].detach().cpu() for k in O.trainable_names(weights)}
    # ff_effnet: the decoder ReLU branches the HIP step took (flip-aware gradient reference, as
    # in test_cfg1_trainer_step_224; the encoder's swish has no branch)
    mh = hip_decoder_relu_masks(eng, weights) if model == "ff_effnet" else None
    del eng, pred, dpred
    torch.cuda.empty_cache()
    P = {k: torch.tensor(v, dtype=torch.float64) for k, v in weights.items()}
    taps = {}
    # ff_redweb: the fp64 / fp32 runs' own ReLU branches (the fp64 one also measures how far
    # from 0 each HIP flip lies)
    b64, b32 = (FlipProbe(mr) if mr is not None else {}), {}
    kw64 = dict(kw, relu_branches=b64) if mr is not None else kw
    pred_ref, loss_ref, dpred_ref, g64 = _oracle_step(
        O, P, torch.tensor(x, dtype=torch.float64), y, B, L, taps=taps, **kw64)
    ref = {n: taps[n].permute(0, 2, 3, 1) for n in names}
    z64 = ({i: taps[f"dec{i}_z"] for i in range(len(mh))} if mh is not None else None)
    del taps
    P32 = {k: torch.tensor(v, dtype=torch.float32) for k, v in weights.items()}
    taps32 = {}
    with torch.no_grad():
        pred32 = O.forward(P32, torch.tensor(x), taps=taps32,
                           **(dict(kw, relu_branches=b32) if mr is not None else kw))
    e32 = {n: rel(taps32[n].permute(0, 2, 3, 1), ref[n]) for n in names}
    e32["pred"] = rel(pred32, pred_ref)
    m32 = ({i: (taps32[f"dec{i}_z"] > 0).double() for i in range(len(mh))}
           if mh is not None else None)
    del taps32, pred32
    g32 = O.train_step_grads(P32, torch.tensor(x), torch.tensor(dpred_ref).float(), **kw)[0]
    errs = {n: rel(hip_taps[n], ref[n]) for n in names}
    errs["pred"] = rel(hip_pred, pred_ref)
    errs["loss"] = abs(hip_loss - loss_ref) / abs(loss_ref)
    bars = {n: max(TOL, 2.0 * e32[n]) for n in e32}
    bars["loss"] = TOL
    report(f"{model}_b32_auto_forward", {"errors": errs, "bars": bars, "fp32_restatement": e32,
                                         "schedule_table_sha1": bench_schedules})
    print(errs, bars)
    assert all(errs[n] < bars[n] for n in errs), (errs, bars)
    if mr is not None:
        # every ReLU of the ResNet encoder and the decoder, flip-aware as ff_effnet's decoder
        x64 = torch.tensor(x, dtype=torch.float64)
        dref = torch.tensor(dpred_ref, dtype=torch.float64)
        flips = {st: {"hip": int((mr[st] != b64[st]).sum()), "fp32": int((b32[st] != b64[st]).sum())}
                 for st in OR.relu_sites()}
        tot = {"hip": sum(v["hip"] for v in flips.values()),
               "fp32": sum(v["fp32"] for v in flips.values())}
        margins = dict(b64.margin)
        margin = assert_flip_margins(margins)
        plain = {k: {"hip": rel(hip_grads[k], g64[k]), "fp32_restatement": rel(g32[k], g64[k])}
                 for k in g64}
        del g64, b64
        g64h = O.train_step_grads(P, x64, dref, relu_masks=mr, **kw)[0]
        g64f = O.train_step_grads(P, x64, dref, relu_masks=b32, **kw)[0]
        second = native_conv_restatement(O, P32, torch.tensor(x), dref.float(), P, x64, dref,
                                         **kw)
        # flip-aware at every ReLU site; the bar from both fp32 restatements (check_gradients)
        check_gradients(f"{model}_b32_auto_grads", hip_grads, g64h, g32, zero, g64_32=g64f,
                        extra={"relu_flips_vs_fp64_total": tot, "relu_flips_vs_fp64": flips,
                               "flip_margin": margins, "flip_margin_check": margin,
                               "plain_comparison": plain}, second=second)
        return
    # each implementation against the fp64 gradient along its own decoder ReLU branches, the
    # strict bar for every tensor (no ill-conditioned exception); the plain comparison and the
    # flip counts go to the report
    x64 = torch.tensor(x, dtype=torch.float64)
    dref = torch.tensor(dpred_ref, dtype=torch.float64)
    flips = {f"dec{i}": {"hip": int(((mh[i] > 0) != (zr > 0)).sum()),
                         "fp32": int(((m32[i] > 0) != (zr > 0)).sum())}
             for i, zr in ((i, z64[i]) for i in range(len(mh)))}
    margins = {f"dec{i}": flip_margin(z64[i], mh[i]) for i in range(len(mh))}
    margin = assert_flip_margins(margins)
    plain = {k: {"hip": rel(hip_grads[k], g64[k]), "fp32_restatement": rel(g32[k], g64[k])}
             for k in g64}
    del g64
    g64h = O.train_step_grads(P, x64, dref, relu_masks=mh)[0]
    g64f = O.train_step_grads(P, x64, dref, relu_masks=m32)[0]
    check_gradients(f"{model}_b32_auto_grads", hip_grads, g64h, g32, zero, g64_32=g64f,
                    extra={"relu_flips_vs_fp64": flips, "flip_margin": margins,
                           "flip_margin_check": margin, "plain_comparison": plain})
