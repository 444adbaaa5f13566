"""ff_effnet on MI355X: EfficientNetB0 encoder (frozen convs, trainable BN) + the PLDepth decoder.

Replaces the Keras graph built by ``EffNetFullyFledged.get_model_and_normalization``
(pldepth/models/pl_hourglass.py:45-100) and the TF kernels Keras dispatches for its forward and
backward passes. Every FLOP runs in libpldepth_hip.so; this module only owns device buffers,
orders the launches on one stream and names parameters after the Keras layers (so weights map
1:1 to the reference's ``model.get_weights()`` layout: Conv2D kernels HWIO, depthwise
[k][k][c], BN gamma/beta/moving_mean/moving_variance).

Data layout in HBM (one replica):
  * ``params``  flat fp32, every trainable tensor (decoder conv kernels + biases, all 54 BN
                gamma/beta) — the Adam / all-reduce unit; ``grads``, Adam m, v, vhat alike;
  * ``frozen``  flat fp32, encoder conv / depthwise / SE weights and the input normalisation;
  * ``stats``   flat fp32, BN moving mean / variance;
  * native copies of every conv filter ([cout][kh][kw][cin] forward, flipped [cin][kh][kw][cout]
    for dX), refreshed after each optimizer step for the trainable (decoder) filters;
  * activations NHWC fp32: every pre-BN tensor is kept for the backward pass (BN and its
    activation are re-applied from it), plus the post-activation tensors the next op reads.
"""
import math
import os

import numpy as np
import torch

from .. import kernels as K
from .engine_common import FlatStore, _BN, _Conv, refresh_trainable_convs  # noqa: F401  (re-exported)

BN_EPS = 1e-3
BN_MOMENTUM = 0.99
# keras.applications.efficientnet DEFAULT_BLOCKS_ARGS (B0): kernel, repeats, in, out, expand, stride
B0_BLOCKS = [
    (3, 1, 32, 16, 1, 1),
    (3, 2, 16, 24, 6, 2),
    (5, 2, 24, 40, 6, 2),
    (3, 3, 40, 80, 6, 2),
    (5, 3, 80, 112, 6, 1),
    (5, 4, 112, 192, 6, 2),
    (3, 1, 192, 320, 6, 1),
]
DROP_CONNECT_RATE = 0.2
# decoder (pl_hourglass.py:59-96): conv name, cout, skip concatenated after the x2 upsampling
DECODER = [
    ("dec_conv0", 672, "block6a_expand_activation"),
    ("dec_conv1", 240, "block4a_expand_activation"),
    ("dec_conv2", 144, "block3a_expand_activation"),
    ("dec_conv3", 32, None),
    ("dec_conv4", 32, None),
]
# Keras' EfficientNet ImageNet checkpoint (TF 2.3-2.8) stores these in its Normalization layer
# encoder activations the decoder concatenates (pl_hourglass.py:66,75,84): materialised
SKIP_TAPS = tuple(skip for _, _, skip in DECODER if skip)

IMAGENET_MEAN = [0.485, 0.456, 0.406]
IMAGENET_VARIANCE = [0.229, 0.224, 0.225]


def block_specs():
    """(name, kernel, stride, filters_in, filters_out, expand_ratio, drop_rate) per block, as
    keras.applications.efficientnet.EfficientNet expands DEFAULT_BLOCKS_ARGS."""
    out, b = [], 0
    total = float(sum(r for _, r, *_ in B0_BLOCKS))
    for i, (k, reps, fin, fout, ex, s) in enumerate(B0_BLOCKS):
        for j in range(reps):
            out.append((f"block{i + 1}{chr(97 + j)}_", k, s if j == 0 else 1,
                        fin if j == 0 else fout, fout, ex, DROP_CONNECT_RATE * b / total))
            b += 1
    return out


def correct_pad(size, k):
    """keras imagenet_utils.correct_pad -> (before, after) for one spatial dim."""
    adjust = 1 - size % 2
    return k // 2 - adjust, k // 2


def same_pad(size, k, s):
    out = -(-size // s)
    total = max((out - 1) * s + k - size, 0)
    return total // 2, out


class EffNetFF:
    """Keras-named parameters + buffers + launch order of one ff_effnet replica."""

    # Keras' automatic names of the decoder layers pl_hourglass.py:59-96 leaves unnamed (a fresh
    # session), for the .h5 import/export (util/keras_h5.py)
    KERAS_RENAME = dict([(f"dec_conv{i}", "conv2d" + (f"_{i}" if i else "")) for i in range(6)]
                        + [(f"dec_bn{i}", "batch_normalization" + (f"_{i}" if i else ""))
                           for i in range(5)])
    # the Normalization layer's adapt() counter, which Keras saves with its mean / variance
    KERAS_EXTRA_WEIGHTS = {"normalization": [("count", np.array(0, np.int64))]}

    def __init__(self, input_shape=(448, 448, 3), batch_size=32, device="cuda", seed=0,
                 conv_math=None):
        H, W, C = input_shape
        # conv arithmetic per part (kernels.conv_policy): encoder / decoder
        self.enc_math, self.dec_math = K.conv_policy(conv_math)
        # per decoder conv index: an arithmetic other than dec_math for its forward / its
        # backward (precision experiments, tools/exp_dec_precision.py)
        self.dec_math_fwd, self.dec_math_bwd = {}, {}
        assert C == 3 and H % 32 == 0 and W % 32 == 0, "input must be RGB with H, W % 32 == 0"
        self.H, self.W, self.B = H, W, batch_size
        self.device = torch.device(device)
        self.params, self.frozen, self.stats = FlatStore(), FlatStore(), FlatStore()
        self.bns, self.convs = [], []
        self._build_spec()
        self.params.materialize(self.device)
        self.grads = self.params.like().materialize(self.device)
        self.frozen.materialize(self.device)
        self.stats.materialize(self.device)
        for m in self.bns + self.convs:
            m.bind(self)
        self.norm_scale = torch.empty(3, device=self.device)
        self.norm_shift = torch.empty(3, device=self.device)
        self.init_weights(seed)
        # thin-N 1x1 convs with the neighbouring BN (+ act, SE gate) folded in (pgemm.hip)
        self.fuse_pgemm = True
        self._alloc_activations()
        self.drop_connect = True
        self.seed = seed
        # training: the last decoder stage's upsample runs inside the final conv's kernels
        # (csrc/upconv.hip); False = the unfused upsample2x + 3x3 conv path
        self.fuse_final = True
        # backward: the decoder convs' weight gradients (dW + bias sums) on a side stream, joined
        # at the end of the backward: 1 = each forked once its layer's pre-BN gradient exists
        # (concurrent with the rest of the decoder chain), 2 = all forked after the last decoder
        # dgrad (concurrent with the encoder backward, which has no weight gradients of its
        # own; +0.7 % img/s, while mode 1 costs 1.5 %: profiles/r03_overlap_ab.txt); 0 = in line
        self.overlap_wgrad = int(os.environ.get("PLD_OVERLAP_WGRAD", "2"))

    # ------------------------------------------------------------------ graph structure
    def _build_spec(self):
        f = self.frozen
        f.add("normalization/mean", (3,))
        f.add("normalization/variance", (3,))
        self.stem = _Conv(self, "stem_conv", 3, 3, 32, stride=2, need_dgrad=False)
        self.stem_bn = _BN(self, "stem_bn", 32)
        self.blocks = []
        for name, k, s, cin, cout, ex, rate in block_specs():
            cexp = cin * ex
            cse = max(1, int(cin * 0.25))
            blk = dict(name=name, k=k, s=s, cin=cin, cout=cout, ex=ex, rate=rate, cexp=cexp,
                       cse=cse, residual=(s == 1 and cin == cout))
            if ex != 1:
                blk["expand"] = _Conv(self, name + "expand_conv", 1, cin, cexp)
                blk["expand_bn"] = _BN(self, name + "expand_bn", cexp)
            blk["dw"] = f.add(name + "dwconv/depthwise_kernel", (k, k, cexp))
            blk["bn"] = _BN(self, name + "bn", cexp)
            blk["se_w1"] = f.add(name + "se_reduce/kernel", (1, 1, cexp, cse))
            blk["se_b1"] = f.add(name + "se_reduce/bias", (cse,))
            blk["se_w2"] = f.add(name + "se_expand/kernel", (1, 1, cse, cexp))
            blk["se_b2"] = f.add(name + "se_expand/bias", (cexp,))
            blk["project"] = _Conv(self, name + "project_conv", 1, cexp, cout)
            blk["project_bn"] = _BN(self, name + "project_bn", cout)
            self.blocks.append(blk)
        self.top = _Conv(self, "top_conv", 1, 320, 1280)
        self.top_bn = _BN(self, "top_bn", 1280)
        self.dec = []
        cin = 1280
        skip_c = {"block6a_expand_activation": 672, "block4a_expand_activation": 240,
                  "block3a_expand_activation": 144}
        for i, (name, cout, skip) in enumerate(DECODER):
            conv = _Conv(self, name, 3, cin, cout, bias=True, trainable=True)
            bn = _BN(self, f"dec_bn{i}", cout)
            self.dec.append((conv, bn, skip))
            cin = cout + (skip_c[skip] if skip else 0)
        self.final = _Conv(self, "dec_conv5", 3, 32, 1, bias=True, trainable=True)

    # ------------------------------------------------------------------ weights
    def init_weights(self, seed=0):
        """Keras default initialisers (ImageNet weights are a network download the reference
        makes at pl_hourglass.py:48; unavailable offline): EfficientNet convs
        VarianceScaling(2.0, fan_out, truncated_normal), decoder Conv2D glorot_uniform, zero
        biases, BN gamma=1 beta=0 mean=0 var=1, ImageNet normalisation constants."""
        rng = np.random.default_rng(seed)
        host = {}

        def trunc_normal(shape, std):
            v = rng.standard_normal(int(np.prod(shape)))
            bad = np.abs(v) > 2
            while bad.any():
                v[bad] = rng.standard_normal(int(bad.sum()))
                bad = np.abs(v) > 2
            return (v * std).reshape(shape)

        def vs_fan_out(shape, depthwise=False):
            k = shape[0] * shape[1]
            fan_out = k * (1 if depthwise else shape[-1])
            return trunc_normal(shape, math.sqrt(2.0 / fan_out) / 0.87962566103423978)

        for name, shape, _ in self.frozen.specs:
            if name == "normalization/mean":
                host[name] = np.array(IMAGENET_MEAN)
            elif name == "normalization/variance":
                host[name] = np.array(IMAGENET_VARIANCE)
            elif name.endswith("/bias"):
                host[name] = np.zeros(shape)
            elif name.endswith("depthwise_kernel"):
                host[name] = vs_fan_out(shape + (1,), depthwise=True).reshape(shape)
            else:
                host[name] = vs_fan_out(shape)
        for name, shape, _ in self.params.specs:
            if name.endswith("/gamma"):
                host[name] = np.ones(shape)
            elif name.endswith("/beta") or name.endswith("/bias"):
                host[name] = np.zeros(shape)
            else:  # decoder conv kernels: glorot_uniform
                rf = shape[0] * shape[1]
                lim = math.sqrt(6.0 / (rf * shape[2] + rf * shape[3]))
                host[name] = rng.uniform(-lim, lim, shape)
        for name, shape, _ in self.stats.specs:
            host[name] = np.ones(shape) if name.endswith("variance") else np.zeros(shape)
        self.set_weights(host)

    def get_weights(self):
        """{keras_name: numpy float32} for every parameter, frozen weight and BN statistic."""
        out = {}
        for store in (self.params, self.frozen, self.stats):
            for name in store.names():
                out[name] = store[name].detach().cpu().numpy().copy()
        return out

    def set_weights(self, weights):
        for store in (self.params, self.frozen, self.stats):
            for name, shape, _ in store.specs:
                if name in weights:
                    store[name].copy_(torch.as_tensor(np.asarray(weights[name], np.float32)
                                                      .reshape(shape)))
        self.refresh_frozen()
        self.refresh_trainable()

    def refresh_frozen(self):
        for c in self.convs:
            if not c.trainable:
                c.refresh()
        # Rescaling(1/255) + Normalization folded into the stem conv's input prologue
        mean = self.frozen["normalization/mean"].double().cpu()
        var = self.frozen["normalization/variance"].double().cpu()
        sd = torch.clamp(torch.sqrt(var), min=1e-7)
        self.norm_scale.copy_((1.0 / (255.0 * sd)).float())
        self.norm_shift.copy_((-mean / sd).float())

    def refresh_trainable(self):
        refresh_trainable_convs(self)

    # ------------------------------------------------------------------ activations
    def _alloc_activations(self):
        B, H, W = self.B, self.H, self.W
        dev = self.device
        self.act, self.gact = {}, {}

        def new(name, shape, grad=True):
            self.act[name] = torch.empty(shape, device=dev)
            if grad:
                self.gact[name] = torch.empty(shape, device=dev)

        new("input", (B, H, W, 3), grad=False)
        h, w = H // 2, W // 2
        new("stem_pre", (B, h, w, 32), grad=False)
        new("stem_activation", (B, h, w, 32))
        for blk in self.blocks:
            n, k, s, cexp, cout = blk["name"], blk["k"], blk["s"], blk["cexp"], blk["cout"]
            blk["h"], blk["w"] = h, w
            if blk["ex"] != 1:
                new(n + "expand_pre", (B, h, w, cexp), grad=False)
                new(n + "expand_activation", (B, h, w, cexp))
            if s == 2:
                pt, _ = correct_pad(h, k)
                pl, _ = correct_pad(w, k)
                oh, ow = h // 2, w // 2
            else:
                pt, oh = same_pad(h, k, 1)
                pl, ow = same_pad(w, k, 1)
            blk["pad"], blk["oh"], blk["ow"] = (pt, pl), oh, ow
            new(n + "dw_pre", (B, oh, ow, cexp), grad=False)
            new(n + "activation", (B, oh, ow, cexp))      # swish(bn(dw)) (SE input)
            new(n + "se_excite", (B, oh, ow, cexp))       # activation * gate
            new(n + "project_pre", (B, oh, ow, cout), grad=False)
            new(n + "output", (B, oh, ow, cout))
            blk["pooled"] = torch.empty(B, cexp, device=dev)
            blk["z1"] = torch.empty(B, blk["cse"], device=dev)
            blk["gate"] = torch.empty(B, cexp, device=dev)
            blk["addn"] = torch.empty(B, cexp, device=dev)
            blk["drop"] = torch.ones(B, device=dev)
            # thin-N 1x1 convs with their neighbouring elementwise op folded in (pgemm.hip):
            # the project conv over BN + swish + SE gate, the expand dgrad over the BN backward
            blk["fused_project"] = self.fuse_pgemm and K.pgemm_pays(cexp, cout)
            blk["fused_expand_dgrad"] = (self.fuse_pgemm and blk["ex"] != 1
                                         and K.pgemm_pays(cexp, blk["cin"]))
            h, w = oh, ow
        # a residual block's output gradient shares its input's gradient buffer: the block's
        # backward reads dy (its project BN backward) before its expand dgrad accumulates onto
        # it, which leaves dy + d(block branch) = d(block input) with no residual-add pass
        prev = None
        for blk in self.blocks:
            if blk["residual"]:
                self.gact[blk["name"] + "output"] = self.gact[prev + "output"]
            prev = blk["name"]
        # drop-connect keep factors of every residual block, one row each (one launch per step)
        self._drop_layers = [li for li, blk in enumerate(self.blocks)
                             if blk["residual"] and blk["rate"] > 0]
        if self._drop_layers:
            self._drop_all = torch.ones(len(self._drop_layers), B, device=dev)
            for s, li in enumerate(self._drop_layers):
                self.blocks[li]["drop"] = self._drop_all[s]
        new("top_pre", (B, h, w, 1280), grad=False)
        new("top_activation", (B, h, w, 1280))
        for i, (conv, bn, skip) in enumerate(self.dec):
            new(f"dec{i}_pre", (B, h, w, conv.cout), grad=False)
            new(f"dec{i}_act", (B, h, w, conv.cout))
            h, w = 2 * h, 2 * w
            new(f"dec{i}_up", (B, h, w, conv.cout))
        new("pred", (B, H, W, 1))
        # pre-BN gradient scratch, one per distinct shape
        self._gpre = {}

    def tap(self, name):
        """An activation by its Keras layer name, materialised on demand where the training
        forward folds it into its consumer (stem_activation: block1a's depthwise prologue)."""
        if name == "stem_activation":
            B, h, w = self.B, self.H // 2, self.W // 2
            self.stem_bn.apply(self.act["stem_pre"], B * h * w, "swish",
                               self.act["stem_activation"], True)
        return self.act[name]

    def _k12_buf(self, c):
        """BN-backward coefficients [2c] (pgemm_bn_bwd's k12), one scratch per width."""
        if not hasattr(self, "_k12"):
            self._k12 = {}
        if c not in self._k12:
            self._k12[c] = torch.empty(2 * c, device=self.device)
        return self._k12[c]

    def _gpre_buf(self, shape, slot=0):
        key = (tuple(shape), slot)
        if key not in self._gpre:
            self._gpre[key] = torch.empty(key[0], device=self.device)
        return self._gpre[key]

    def _wgrad_side(self):
        """(stream, fork events) of the decoder's weight-gradient side stream (created once)."""
        if not hasattr(self, "_wside"):
            self._wside = (torch.cuda.Stream(device=self.device),
                           [torch.cuda.Event() for _ in range(len(self.dec) + 1)])
        return self._wside

    # ------------------------------------------------------------------ forward
    def _em(self, oh, ow):
        """Encoder conv math for a conv with an oh x ow output (its BN sees B*oh*ow values)."""
        return K.encoder_math(self.enc_math, self.B * oh * ow)

    def forward(self, training=True, step=0, image_offset=0):
        """step: int or device int64 tensor (drop-connect Philox counter); image_offset: global
        index of this replica's first image (draws independent of the GPU count)."""
        self._img_off = image_offset
        A = self.act
        B = self.B
        a = K.conv_args
        # stem: normalisation prologue, TF-SAME stride-2 (correct_pad) conv, BN, swish
        pt, _ = correct_pad(self.H, 3)
        pl, _ = correct_pad(self.W, 3)
        x = A["input"]
        h, w = self.H // 2, self.W // 2
        rows = B * h * w
        args = a(x, None, 3, 3, 2, pt, pl, h, w, 32, self.norm_scale, self.norm_shift, "none",
                 math=self._em(h, w))
        self._conv_bn(args, self.stem.w_nat, None, A["stem_pre"], self.stem_bn, rows, training)
        if training:
            # stem BN + swish applied by block1a's depthwise conv as it reads its taps: the stem
            # activation (its only consumer in training) is never materialised
            x = None
        else:
            self.stem_bn.apply(A["stem_pre"], rows, "swish", A["stem_activation"], training)
            x = A["stem_activation"]
        if training and self.drop_connect and self._drop_layers:
            K.dropconnect_scales_multi(self._drop_all,
                                       [self.blocks[li]["rate"] for li in self._drop_layers],
                                       self._drop_layers, self.seed, step, image_offset)
        for li, blk in enumerate(self.blocks):
            x = self._block_fwd(blk, x, training, step, li)
        h, w = x.shape[1], x.shape[2]
        rows = B * h * w
        self.top_bn.conv_fwd_stats(a(x, None, 1, 1, 1, 0, 0, h, w, 1280, math=self._em(h, w)),
                                   self.top.w_nat, None, A["top_pre"], rows, training)
        self.top_bn.apply(A["top_pre"], rows, "swish", A["top_activation"], training)
        x, x2 = A["top_activation"], None
        for i, (conv, bn, skip) in enumerate(self.dec):
            pt, _ = same_pad(h, 3, 1)
            pl, _ = same_pad(w, 3, 1)
            args = a(x, x2, 3, 3, 1, pt, pl, h, w, conv.cout,
                     math=self.dec_math_fwd.get(i, self.dec_math))
            rows = B * h * w
            bn.conv_fwd_stats(args, conv.w_nat, conv.b, A[f"dec{i}_pre"], rows, training)
            if training and i == len(self.dec) - 1 and self.fuse_final:
                pass  # BN + ReLU + upsample folded into the final conv (upconv_fwd below)
            elif training:
                # BN + ReLU applied as the upsampling reads its taps: dec{i}_act is never
                # materialised (backward re-derives it from dec{i}_pre)
                K.upsample2x_fwd(A[f"dec{i}_pre"], A[f"dec{i}_up"],
                                 bn=(bn.mean, bn.invstd, bn.gamma, bn.beta), act="relu")
            else:
                bn.apply(A[f"dec{i}_pre"], rows, "relu", A[f"dec{i}_act"], training)
                K.upsample2x_fwd(A[f"dec{i}_act"], A[f"dec{i}_up"])
            h, w = 2 * h, 2 * w
            x, x2 = A[f"dec{i}_up"], (A[skip] if skip else None)
        if training and self.fuse_final:
            # dec_conv5(up(relu(bn4(dec4_pre)))): the 448^2 x 32 map is never written
            _, bn4, _ = self.dec[-1]
            K.upconv_fwd(A["dec4_pre"], (bn4.mean, bn4.invstd, bn4.gamma, bn4.beta),
                         self.final.w_nat, self.final.b, A["pred"])
            return A["pred"]
        pt, _ = same_pad(h, 3, 1)
        pl, _ = same_pad(w, 3, 1)
        K.conv2d_fwd(a(x, None, 3, 3, 1, pt, pl, h, w, 1, math=self.dec_math), self.final.w_nat,
                     self.final.b, A["pred"])
        return A["pred"]

    def _block_fwd(self, blk, x, training, step, li):
        A, B, n = self.act, self.B, blk["name"]
        h, w, oh, ow = blk["h"], blk["w"], blk["oh"], blk["ow"]
        pt, pl = blk["pad"]
        bn = blk["bn"]
        rows = B * oh * ow
        dwk = (self.frozen[blk["dw"]], blk["k"], blk["s"], pt, pl)
        if blk["ex"] != 1:
            ebn = blk["expand_bn"]
            self._conv_bn(K.conv_args(x, None, 1, 1, 1, 0, 0, h, w, blk["cexp"],
                                      math=self._em(h, w)),
                          blk["expand"].w_nat, None, A[n + "expand_pre"], ebn, B * h * w,
                          training)
            if training and n + "expand_activation" not in SKIP_TAPS:
                # BN + swish fused into the depthwise conv's input read: the activation is
                # never materialised (only the decoder's skip taps need it)
                src, pro = A[n + "expand_pre"], ebn
            else:
                ebn.apply(A[n + "expand_pre"], B * h * w, "swish", A[n + "expand_activation"],
                          training)
                src, pro = A[n + "expand_activation"], None
        elif x is None:  # block1a in training: the stem's pre-BN output through BN + swish
            src, pro = A["stem_pre"], self.stem_bn
        else:
            src, pro = x, None
        bnp = (pro.mean, pro.invstd, pro.gamma, pro.beta) if pro is not None else None
        if training:
            # the depthwise output's BN statistics gathered in the tiled kernel's epilogue
            K.dwconv_fwd_bn_stats(src, *dwk, A[n + "dw_pre"],
                                  (bn.mean, bn.invstd, bn.mmean, bn.mvar), bn=bnp,
                                  act="swish" if pro is not None else "none", eps=bn.eps,
                                  momentum=bn.momentum)
        else:
            K.dwconv_fwd(src, *dwk, A[n + "dw_pre"], bn=bnp,
                         act="swish" if pro is not None else "none")
            bn.stats_(A[n + "dw_pre"], rows, training)
        F = self.frozen
        se_w = (F[blk["se_w1"]].view(blk["cexp"], blk["cse"]), F[blk["se_b1"]],
                F[blk["se_w2"]].view(blk["cse"], blk["cexp"]), F[blk["se_b2"]])
        pg = training and blk["fused_project"]
        if pg:
            # the SE squeeze applies BN + swish to dw_pre on the fly, and the project conv reads
            # dw_pre through BN + swish + the SE gate (pgemm): neither the block's activation
            # nor se_excite is materialised
            K.se_fwd(A[n + "dw_pre"], *se_w, blk["pooled"], blk["z1"], blk["gate"],
                     bn=(bn.mean, bn.invstd, bn.gamma, bn.beta), act="swish")
            K.pgemm_bn_act(A[n + "dw_pre"], rows, blk["cexp"], bn.mean, bn.invstd, bn.gamma,
                           bn.beta, "swish", blk["project"].w_nat, blk["cout"],
                           A[n + "project_pre"], gate=blk["gate"], hw=oh * ow)
        else:
            if training:
                # the SE squeeze applies BN + swish to dw_pre on the fly and se_excite is written
                # straight from dw_pre: the block's activation is never materialised
                K.se_fwd(A[n + "dw_pre"], *se_w, blk["pooled"], blk["z1"], blk["gate"],
                         bn=(bn.mean, bn.invstd, bn.gamma, bn.beta), act="swish")
                bn.apply(A[n + "dw_pre"], rows, "swish", A[n + "se_excite"], True,
                         gate=blk["gate"], hw=oh * ow)
            else:
                bn.apply(A[n + "dw_pre"], rows, "swish", A[n + "activation"], training)
                K.se_fwd(A[n + "activation"], *se_w, blk["pooled"], blk["z1"], blk["gate"])
                self._gate_mul(A[n + "activation"], blk["gate"], A[n + "se_excite"])
        pbn = blk["project_bn"]
        if pg:
            pbn.stats_(A[n + "project_pre"], rows, training)
        else:
            pbn.conv_fwd_stats(K.conv_args(A[n + "se_excite"], None, 1, 1, 1, 0, 0, oh, ow,
                                           blk["cout"], math=self._em(oh, ow)),
                               blk["project"].w_nat, None, A[n + "project_pre"], rows, training)
        out = A[n + "output"]
        if blk["residual"] and training:
            # project BN -> drop-connect -> + block input in one pass (pld_bn_scale_add_apply)
            drop = None
            if self.drop_connect and blk["rate"] > 0:
                drop = blk["drop"]  # this step's keep factors (forward: one launch, all blocks)
            K.bn_scale_add_apply(A[n + "project_pre"], rows, blk["cout"], pbn.mean, pbn.invstd,
                                 pbn.gamma, pbn.beta, drop, oh * ow, x, "none", out)
            return out
        pbn.apply(A[n + "project_pre"], rows, "none", out, training)
        if blk["residual"]:
            K.residual_add(out, None, x, out)
        return out

    def _conv_bn(self, args, w_nat, bias, out, bn, rows, training):
        """conv forward + the batch statistics of its output for the BN after it (training: in
        the conv's epilogue where its kernel supports it; inference: the moving statistics)."""
        if training:
            K.conv2d_fwd_bn_stats(args, w_nat, bias, out, bn.mean, bn.invstd, bn.mmean, bn.mvar,
                                  bn.eps, bn.momentum)
        else:
            K.conv2d_fwd(args, w_nat, bias, out)
            bn.stats_(out, rows, training)

    def _gate_mul(self, a, gate, y):
        """inference path: y = a * gate[img][c] (a BN apply with identity statistics is exact:
        ((a - 0) * 1) * 1 + 0 = a, then * gate)."""
        c = a.shape[-1]
        if not hasattr(self, "_ident"):
            self._ident = {}
        if c not in self._ident:
            self._ident[c] = (torch.zeros(c, device=self.device),
                              torch.ones(c, device=self.device))
        z, o = self._ident[c]
        K.bn_apply(a, a.numel() // c, c, z, o, o, z, "none", y, gate=gate,
                   hw=a.shape[1] * a.shape[2])

    # ------------------------------------------------------------------ backward
    def param_offset(self, name):
        """Offset of a trainable tensor in the flat params / grads buffers."""
        return next(off for n, _, off in self.params.specs if n == name)

    def backward(self, dpred):
        """Backward from d loss / d pred: fills self.grads (decoder kernels/biases, BN params).
        The decoder chain (backward_decoder), its deferred weight gradients on the side stream
        beside the encoder chain (backward_encoder), joined at the end."""
        deferred = self.backward_decoder(dpred)
        main = torch.cuda.current_stream(self.device)
        if deferred:
            wstream, fork = self._wgrad_side()
            fork[-1].record(main)
            with torch.cuda.stream(wstream):
                wstream.wait_event(fork[-1])
                for wg in deferred:
                    wg()
        self.backward_encoder()
        if self.overlap_wgrad:  # join: every weight gradient is final on the caller's stream
            main.wait_stream(self._wgrad_side()[0])

    def backward_decoder(self, dpred):
        """The decoder part of the backward on the current stream, down to the gradient of the
        encoder's top activation. Returns the weight-gradient calls deferred for the side stream
        (overlap_wgrad == 2; [] otherwise: run inline, or forked per layer in mode 1). Split out
        so that the data-parallel trainer can all-reduce the decoder's gradients while the
        encoder's backward runs (ReplicaTrainer.dp_overlap)."""
        A, G, B = self.act, self.gact, self.B
        a = K.conv_args
        h, w = self.H, self.W
        # the side stream needs its own buffers: gradients it reads are never recycled by the
        # main stream's later layers (slot "dec"), its bias sums use their own workspace
        side = bool(self.overlap_wgrad)
        main = torch.cuda.current_stream(self.device)
        if side:
            wstream, fork = self._wgrad_side()
            deferred = []
        # final conv (bias, no BN)
        last = len(self.dec) - 1
        if self.fuse_final:
            # through the fused upsample, one pass over (dec4_pre, dpred): the filter gradient,
            # dec4's activation gradient and the whole dec_bn4 + ReLU backward (its channel
            # reductions accumulated in the same pass) into dec4's pre-BN gradient
            _, bn4, _ = self.dec[last]
            gpre4 = self._gpre_buf(A[f"dec{last}_pre"].shape, "dec" if side else 0)
            K.upconv_bwd(A["dec4_pre"], (bn4.mean, bn4.invstd, bn4.gamma, bn4.beta),
                         self.final.w_nat, dpred, G[f"dec{last}_act"], dw=self.final.dw,
                         dx=gpre4, dgamma=bn4.dgamma, dbeta=bn4.dbeta)
            K.channel_sum(dpred, B * h * w, 1, self.final.db)
        else:
            pt, _ = same_pad(h, 3, 1)
            pl, _ = same_pad(w, 3, 1)
            x4 = A["dec4_up"]
            args = a(x4, None, 3, 3, 1, pt, pl, h, w, 1, math=self.dec_math)
            K.conv2d_wgrad(args, dpred, self.final.dw)
            K.channel_sum(dpred, B * h * w, 1, self.final.db)
            K.conv2d_dgrad(args, dpred, self.final.w_dg, G["dec4_up"])
        # after the layer's dgrad: its filter copies are no longer read this step (a caller
        # may update and refresh them from here on)
        for i in range(len(self.dec) - 1, -1, -1):
            conv, bn, skip = self.dec[i]
            h, w = h // 2, w // 2
            if not (i == last and self.fuse_final):
                K.upsample2x_bwd(G[f"dec{i}_up"], G[f"dec{i}_act"])
            rows = B * h * w
            gpre = self._gpre_buf(A[f"dec{i}_pre"].shape, "dec" if side else 0)
            if not (i == last and self.fuse_final):  # (fused: done by upconv_bwd above)
                bn.bwd(A[f"dec{i}_pre"], G[f"dec{i}_act"], rows, "relu", gpre)
            if i == 0:
                x1, x2, g1, g2 = A["top_activation"], None, G["top_activation"], None
            else:
                pconv, _, pskip = self.dec[i - 1]
                x1 = A[f"dec{i - 1}_up"]
                x2 = A[pskip] if pskip else None
                g1, g2 = G[f"dec{i - 1}_up"], (G[pskip] if pskip else None)
            pt, _ = same_pad(h, 3, 1)
            pl, _ = same_pad(w, 3, 1)
            args = a(x1, x2, 3, 3, 1, pt, pl, h, w, conv.cout,
                     math=self.dec_math_bwd.get(i, self.dec_math))
            if side:
                def wg(args=args, gpre=gpre, rows=rows, conv=conv):
                    K.conv2d_wgrad(args, gpre, conv.dw)
                    K.channel_sum(gpre, rows, conv.cout, conv.db, ws_key="reduce_side")
                if self.overlap_wgrad == 2:
                    deferred.append(wg)
                else:
                    fork[i].record(main)
                    with torch.cuda.stream(wstream):
                        wstream.wait_event(fork[i])
                        wg()
            else:
                K.conv2d_wgrad(args, gpre, conv.dw)
                K.channel_sum(gpre, rows, conv.cout, conv.db)
            K.conv2d_dgrad(args, gpre, conv.w_dg, g1, g2)  # skip grads: fresh write
        return deferred if side else []

    def backward_encoder(self):
        """The encoder part of the backward (after backward_decoder) on the current stream."""
        A, G, B = self.act, self.gact, self.B
        a = K.conv_args
        h, w = A["top_pre"].shape[1:3]
        rows = B * h * w
        gpre = self._gpre_buf(A["top_pre"].shape)
        self.top_bn.bwd(A["top_pre"], G["top_activation"], rows, "swish", gpre)
        last = self.blocks[-1]["name"] + "output"
        K.conv2d_dgrad(a(A[last], None, 1, 1, 1, 0, 0, h, w, 1280, math=self._em(h, w)), gpre,
                       self.top.w_dg, G[last])
        for bi in range(len(self.blocks) - 1, -1, -1):
            blk = self.blocks[bi]
            x_in = A[self.blocks[bi - 1]["name"] + "output"] if bi > 0 else A["stem_activation"]
            gx_in = G[self.blocks[bi - 1]["name"] + "output"] if bi > 0 else G["stem_activation"]
            self._block_bwd(blk, x_in, gx_in)
        rows = B * A["stem_pre"].shape[1] * A["stem_pre"].shape[2]
        self.stem_bn.bwd(A["stem_pre"], G["stem_activation"], rows, "swish", None)

    def _block_bwd(self, blk, x_in, gx_in):
        A, G, B, n = self.act, self.gact, self.B, blk["name"]
        h, w, oh, ow = blk["h"], blk["w"], blk["oh"], blk["ow"]
        rows = B * oh * ow
        gy = G[n + "output"]
        drop = None
        if blk["residual"] and self.drop_connect and blk["rate"] > 0:
            drop = blk["drop"]
        gp = self._gpre_buf(A[n + "project_pre"].shape)
        pbn = blk["project_bn"]
        if drop is not None:  # the BN backward of dy * drop (no scaled copy of dy)
            K.bn_bwd_scaled(A[n + "project_pre"], gy, rows, pbn.c, pbn.mean, pbn.invstd,
                            pbn.gamma, pbn.beta, "none", drop, oh * ow, gp, pbn.dgamma,
                            pbn.dbeta)
        else:
            pbn.bwd(A[n + "project_pre"], gy, rows, "none", gp)
        gse = G[n + "se_excite"]
        K.conv2d_dgrad(K.conv_args(A[n + "se_excite"], None, 1, 1, 1, 0, 0, oh, ow, blk["cout"],
                                   math=self._em(oh, ow)),
                       gp, blk["project"].w_dg, gse)
        F = self.frozen
        bn = blk["bn"]
        gdw = self._gpre_buf(A[n + "dw_pre"].shape)
        # SE backward + the block BN's backward; the BN reductions ride on the SE squeeze sweep
        K.se_bwd_bn_full(gse, A[n + "dw_pre"], (bn.mean, bn.invstd, bn.gamma, bn.beta),
                         F[blk["se_w1"]].view(blk["cexp"], blk["cse"]),
                         F[blk["se_w2"]].view(blk["cse"], blk["cexp"]), blk["z1"], blk["gate"],
                         blk["addn"], gdw, bn.dgamma, bn.dbeta, act="swish")
        pt, pl = blk["pad"]
        if blk["ex"] != 1:
            ge = G[n + "expand_activation"]
            # skip taps already hold the decoder's gradient: accumulate onto it
            is_tap = n + "expand_activation" in SKIP_TAPS
            ebn = blk["expand_bn"]
            bnp = (ebn.mean, ebn.invstd, ebn.gamma, ebn.beta)
            k12 = self._k12_buf(blk["cexp"])
            K.dwconv_dgrad(gdw, F[blk["dw"]], blk["k"], blk["s"], pt, pl, ge, accumulate=is_tap)
            # residual: gx_in is gy's buffer (_alloc_activations) and already holds gy
            res = blk["residual"]
            if blk["fused_expand_dgrad"]:
                K.bn_bwd_coeffs(A[n + "expand_pre"], ge, B * h * w, blk["cexp"], *bnp, "swish",
                                ebn.dgamma, ebn.dbeta, k12)
                K.pgemm_bn_bwd(A[n + "expand_pre"], ge, B * h * w, blk["cexp"], *bnp, "swish",
                               k12, blk["expand"].w_dg, blk["cin"], gx_in, accumulate=res)
            else:
                gpe = self._gpre_buf(A[n + "expand_pre"].shape)
                ebn.bwd(A[n + "expand_pre"], ge, B * h * w, "swish", gpe)
                K.conv2d_dgrad(K.conv_args(x_in, None, 1, 1, 1, 0, 0, h, w, blk["cexp"],
                                           math=self._em(h, w)), gpe, blk["expand"].w_dg, gx_in,
                               acc1=res)
        else:
            assert not blk["residual"]
            K.dwconv_dgrad(gdw, F[blk["dw"]], blk["k"], blk["s"], pt, pl, gx_in)

    # ------------------------------------------------------------------ optimizer
    def adam_state(self):
        if not hasattr(self, "_adam"):
            self._adam = [torch.zeros_like(self.params.buf) for _ in range(3)]
        return self._adam

    def adam_step(self, lr, step, grad_scale=1.0, beta1=0.9, beta2=0.999, eps=1e-7):
        m, v, vh = self.adam_state()
        K.adam_amsgrad(self.params.buf, self.grads.buf, m, v, vh, lr, step, beta1, beta2, eps,
                       grad_scale)
        self.refresh_trainable()

    # ------------------------------------------------------------------ counts
    def count_trainable(self):
        return sum(int(np.prod(s)) for _, s, _ in self.params.specs)

    def conv_flops_per_image(self):
        """Algorithmic dense-conv FLOPs per image of one train step (fwd + dX; dW for the
        trainable decoder; no stem dX), the SURVEY §8d accounting."""
        H, W = self.H, self.W
        f = 0.0

        def macs(h, w, k, cin, cout):
            return h * w * k * k * cin * cout

        h, w = H // 2, W // 2
        f += macs(h, w, 3, 3, 32)  # stem fwd only
        for blk in self.blocks:
            if blk["ex"] != 1:
                f += 2 * macs(blk["h"], blk["w"], 1, blk["cin"], blk["cexp"])
            f += 2 * macs(blk["oh"], blk["ow"], 1, blk["cexp"], blk["cout"])
        hh, ww = blk["oh"], blk["ow"]
        f += 2 * macs(hh, ww, 1, 320, 1280)
        cin = 1280
        for conv, _, skip in self.dec:
            f += 3 * macs(hh, ww, 3, conv.cin, conv.cout)
            hh, ww = 2 * hh, 2 * ww
        f += 3 * macs(hh, ww, 3, 32, 1)
        return 2.0 * f
