"""ff_redweb on MI355X: ResNet-50 encoder (frozen convs, trainable BN) + the ReDWeb decoder.

Replaces the Keras graph built by ``ReDWebNetTFVersion.get_model_and_normalization``
(pldepth/models/redweb.py:402-434) — keras.applications ResNet50(include_top=False) tapped at
conv2_block3_out / conv3_block4_out / conv4_block3_out / conv5_block3_out (:418-421), three
FeatureFusionLayers (:225-290, each two BottleneckConvLayers :67-165) and the
AdaptiveOutputLayer (:293-338) — and the TF kernels its forward and backward passes dispatch.
Every FLOP runs in libpldepth_hip.so; this module owns device buffers and launch order.

Parameters carry Keras names (encoder: ResNet50 layer names; decoder: ffl{i}/..., aol/...; see
oracle/redweb.py for the full list), Conv2D kernels HWIO. Encoder convs keep their biases (Keras
ResNet50 convs have use_bias=True) and are frozen like every non-BN encoder layer
(redweb.py:412-416); all BNs and the decoder train. BN epsilon: 1.001e-5 in ResNet50, the Keras
default 1e-3 in the decoder.

Layout in HBM (one replica): flat ``params`` / ``grads`` / Adam state (8,647,299 trainable at any
input size), flat ``frozen`` (encoder kernels + biases), flat ``stats`` (moving mean/variance),
native filter copies per conv, NHWC fp32 activations: each pre-BN tensor (BN backward re-reads
it), each post-activation tensor a later op reads, and one gradient buffer per activation.
The encoder convs need dX only (frozen), the stem conv neither dX nor dW.
"""
import math
import os

import numpy as np
import torch

from .. import kernels as K
from .engine_common import FlatStore, _BN, _Conv, refresh_trainable_convs

RESNET_BN_EPS = 1.001e-5
CAFFE_MEAN_BGR = np.array([103.939, 116.779, 123.68], np.float32)
RESNET50_STACKS = [("conv2", 64, 3, 1), ("conv3", 128, 4, 2), ("conv4", 256, 6, 2),
                   ("conv5", 512, 3, 2)]
TAPS = ("conv2_block3_out", "conv3_block4_out", "conv4_block3_out", "conv5_block3_out")
# FeatureFusionLayer(inter, out)([left tap, up]) (redweb.py:426-428)
# 'auto' conv policy for the frozen ResNet-50: bf16x3 everywhere except the conv2 stage (the
# 112x112 bottlenecks at 448x448), which runs exact fp32. The random-init ResNet-50 under
# training-mode BN amplifies a perturbation ~100x from conv2_block3_out to conv5_block3_out:
# bf16x3 rounding entering in the conv2 stage alone puts conv5_block3_out 1.2e-3 from fp64
# (batch 32, 448x448), with that stage exact it is at the fp32 restatement's own 5e-4;
# exact stem / conv3-5 stages change nothing measurable. Cost: +1.8 ms per fwd+bwd
# (36.9 -> 38.7 ms eager; tools/exp_redweb_policy.py, profiles/r03_redweb_policy.txt).
# Only the FORWARD convs of those stages need it: the activations' rounding is what the chaotic
# encoder amplifies; the backward's dX convs of the frozen encoder run bf16x3 (their ~2^-16
# per-product error sits far below the fp32 restatement's own gradient error, ~5e-2 per tensor
# at batch 32).
EXACT_STAGES_AUTO = ("conv2",)
# Backward (dX / dW) convs kept exact under 'auto' (name prefixes; encoder or decoder).
EXACT_BWD_AUTO = ()
FFLS = [("ffl0", 256, 256, "conv4_block3_out"),
        ("ffl1", 128, 128, "conv3_block4_out"),
        ("ffl2", 64, 64, "conv2_block3_out")]


def preprocess_input(x):
    """keras.applications.resnet50.preprocess_input ('caffe'): RGB->BGR, minus ImageNet means —
    applied by the data pipeline to the [0,1] images (PLDepth.py:169-173)."""
    x = np.asarray(x, np.float32)[..., ::-1]
    return np.ascontiguousarray(x - CAFFE_MEAN_BGR)


class RedWebFF:
    """Keras-named parameters + buffers + launch order of one ff_redweb replica."""

    def __init__(self, input_shape=(448, 448, 3), batch_size=32, device="cuda", seed=0,
                 conv_math=None):
        H, W, C = input_shape
        # conv arithmetic (kernels.conv_policy): frozen ResNet-50 encoder / trainable decoder
        self.enc_math, self.dec_math = K.conv_policy(conv_math)
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
        self.init_weights(seed)
        self._alloc()
        self.drop_connect = False  # no drop-connect in ResNet50 / ReDWeb
        # encoder convs (by Keras name prefix) kept in exact fp32 under the 'auto' policy
        self.exact_stages = EXACT_STAGES_AUTO
        # name prefixes of convs (encoder or decoder) run exact fp32 in the backward / the
        # forward under 'auto' besides exact_stages (RedWebFF._math)
        self.exact_bwd = EXACT_BWD_AUTO
        self.exact_fwd_extra = ()
        # backward: trainable convs' dW + db on a side stream (EffNetFF.overlap_wgrad)
        self.overlap_wgrad = int(os.environ.get("PLD_OVERLAP_WGRAD", "2"))
        # forward: each feature-fusion layer's left branch (conv0 + bn0 + block_left: it reads
        # only its encoder tap) on a side stream, forked as soon as the tap exists, so it runs
        # beside the deeper encoder stages and the decoder layers above it (PLD_OVERLAP_FFL=0:
        # one stream); PLD_OVERLAP_PROJ: the encoder's projection shortcuts (conv0 + bn0 of each
        # stage's first block) beside conv1 -> conv2 -> conv3 in the forward
        self.overlap_ffl = int(os.environ.get("PLD_OVERLAP_FFL", "1"))
        self.overlap_proj = int(os.environ.get("PLD_OVERLAP_PROJ", "1"))
        self._side = False
        self._in_fside = False
        self.seed = seed

    preprocess = staticmethod(preprocess_input)

    # ------------------------------------------------------------------ structure
    def _build_spec(self):
        rbn = lambda name, c: _BN(self, name, c, eps=RESNET_BN_EPS)
        self.stem = _Conv(self, "conv1_conv", 7, 3, 64, stride=2, bias=True, need_dgrad=False)
        self.stem_bn = rbn("conv1_bn", 64)
        self.blocks = []
        cin = 64
        for name, f, nb, s1 in RESNET50_STACKS:
            for b in range(1, nb + 1):
                pre = f"{name}_block{b}_"
                s = s1 if b == 1 else 1
                blk = dict(name=pre, cin=cin, f=f, s=s, proj=(b == 1))
                if b == 1:
                    blk["c0"] = _Conv(self, pre + "0_conv", 1, cin, 4 * f, stride=s, bias=True)
                    blk["bn0"] = rbn(pre + "0_bn", 4 * f)
                blk["c1"] = _Conv(self, pre + "1_conv", 1, cin, f, stride=s, bias=True)
                blk["bn1"] = rbn(pre + "1_bn", f)
                blk["c2"] = _Conv(self, pre + "2_conv", 3, f, f, bias=True)
                blk["bn2"] = rbn(pre + "2_bn", f)
                blk["c3"] = _Conv(self, pre + "3_conv", 1, f, 4 * f, bias=True)
                blk["bn3"] = rbn(pre + "3_bn", 4 * f)
                self.blocks.append(blk)
                cin = 4 * f
        self.ffls = []
        up_c = 2048
        tap_c = {"conv4_block3_out": 1024, "conv3_block4_out": 512, "conv2_block3_out": 256}
        for name, inter, outp, tap in FFLS:
            d = dict(name=name, inter=inter, out=outp, tap=tap)
            d["conv0"] = _Conv(self, name + "/conv0", 3, tap_c[tap], inter, trainable=True)
            d["bn0"] = _BN(self, name + "/bn0", inter)
            d["conv1"] = _Conv(self, name + "/conv1", 3, up_c, inter, trainable=True)
            d["bn1"] = _BN(self, name + "/bn1", inter)
            d["left"] = self._bottleneck_spec(name + "/block_left", inter)
            d["down"] = self._bottleneck_spec(name + "/block_down", outp)
            self.ffls.append(d)
            up_c = outp
        self.aol0 = _Conv(self, "aol/conv0", 3, 64, 64, bias=True, trainable=True)
        self.aol_bn = _BN(self, "aol/bn0", 64)
        self.aol1 = _Conv(self, "aol/conv1", 3, 64, 1, bias=True, trainable=True)
        self.aol2 = _Conv(self, "aol/conv2", 1, 1, 1, bias=True, trainable=True)

    def _bottleneck_spec(self, name, p):
        q = p // 4
        convs, bns = [], []
        for i, (k, ci, co) in enumerate([(1, p, q), (3, q, q), (1, q, p)] * 2):
            convs.append(_Conv(self, f"{name}/conv{i}", k, ci, co, trainable=True))
            bns.append(_BN(self, f"{name}/bn{i}", co))
        return dict(name=name, p=p, q=q, convs=convs, bns=bns)

    # ------------------------------------------------------------------ weights
    def init_weights(self, seed=0):
        """Keras defaults (ImageNet weights are a network download the reference makes at
        redweb.py:410; unavailable offline): Conv2D glorot_uniform kernels and zero biases, BN
        gamma=1 beta=0 moving mean 0 / variance 1."""
        rng = np.random.default_rng(seed)
        host = {}
        for store in (self.frozen, self.params):
            for name, shape, _ in store.specs:
                if name.endswith("/gamma"):
                    host[name] = np.ones(shape)
                elif name.endswith("/beta") or name.endswith("/bias"):
                    host[name] = np.zeros(shape)
                else:
                    rf = shape[0] * shape[1]
                    lim = math.sqrt(6.0 / (rf * shape[2] + rf * shape[3]))
                    host[name] = rng.uniform(-lim, lim, shape)
        for name, shape, _ in self.stats.specs:
            host[name] = np.ones(shape) if name.endswith("variance") else np.zeros(shape)
        self.set_weights(host)

    def get_weights(self):
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
        for c in self.convs:
            c.refresh()

    def refresh_trainable(self):
        refresh_trainable_convs(self)

    # ------------------------------------------------------------------ activations
    def _alloc(self):
        B, H, W, dev = self.B, self.H, self.W, self.device
        self.act, self.gact = {}, {}

        def new(name, shape, grad=True):
            self.act[name] = torch.empty(shape, device=dev)
            if grad:
                self.gact[name] = torch.empty(shape, device=dev)

        new("input", (B, H, W, 3), grad=False)
        h, w = H // 2, W // 2
        new("conv1_pre", (B, h, w, 64), grad=False)
        new("conv1_relu", (B, h, w, 64))
        h, w = h // 2, w // 2
        new("pool1_pool", (B, h, w, 64))
        self.pool_argmax = torch.empty((B, h, w, 64), dtype=torch.uint8, device=dev)
        for blk in self.blocks:
            n, f, s = blk["name"], blk["f"], blk["s"]
            oh, ow = h // s, w // s
            blk["hw"] = (h, w, oh, ow)
            if blk["proj"]:
                new(n + "0_pre", (B, oh, ow, 4 * f), grad=False)
                new(n + "0_bn", (B, oh, ow, 4 * f))
            new(n + "1_pre", (B, oh, ow, f), grad=False)
            new(n + "1_relu", (B, oh, ow, f))
            new(n + "2_pre", (B, oh, ow, f), grad=False)
            new(n + "2_relu", (B, oh, ow, f))
            new(n + "3_pre", (B, oh, ow, 4 * f), grad=False)
            new(n + "out", (B, oh, ow, 4 * f))
            h, w = oh, ow
        new("conv5_up", (B, 2 * h, 2 * w, 2048))
        h, w = 2 * h, 2 * w
        for d in self.ffls:
            n, inter, outp = d["name"], d["inter"], d["out"]
            d["hw"] = (h, w)
            new(n + "/left_pre", (B, h, w, inter), grad=False)
            new(n + "/left_bn", (B, h, w, inter))
            self._bottleneck_alloc(new, d["left"], h, w)
            new(n + "/up_pre", (B, h, w, inter), grad=False)
            new(n + "/sum", (B, h, w, inter))
            self._bottleneck_alloc(new, d["down"], h, w)
            new(n + "/out", (B, 2 * h, 2 * w, outp))
            h, w = 2 * h, 2 * w
        new("aol/pre0", (B, h, w, 64), grad=False)
        new("aol/act0", (B, h, w, 64))
        new("aol/pre1", (B, h, w, 1))
        new("aol/up", (B, 2 * h, 2 * w, 1))
        new("pred", (B, H, W, 1))
        self._gpre = {}

    def _bottleneck_alloc(self, new, bt, h, w):
        B, n, p, q = self.B, bt["name"], bt["p"], bt["q"]
        for half in (0, 3):
            new(f"{n}/pre{half}", (B, h, w, q), grad=False)
            new(f"{n}/act{half}", (B, h, w, q))
            new(f"{n}/pre{half + 1}", (B, h, w, q), grad=False)
            new(f"{n}/act{half + 1}", (B, h, w, q))
            new(f"{n}/pre{half + 2}", (B, h, w, p), grad=False)
            new(f"{n}/out{half}", (B, h, w, p))

    def _gpre_buf(self, shape, slot=0):
        key = (tuple(shape), slot)
        if key not in self._gpre:
            self._gpre[key] = torch.empty(key[0], device=self.device)
        return self._gpre[key]

    # ------------------------------------------------------------------ forward
    def _math(self, conv, oh=None, ow=None, bwd=False):
        if self.enc_math in ("auto", "fp32"):  # 'auto' and 'mixed'
            exact = self.exact_bwd if bwd else self.exact_stages + tuple(self.exact_fwd_extra)
            if exact and conv.name.startswith(tuple(exact)):
                return "fp32"
        if conv.trainable:
            return self.dec_math
        # "auto": per conv by the population its BN normalises over (kernels.encoder_math)
        return K.encoder_math(self.enc_math, self.B * (oh or 1) * (ow or 1),
                              getattr(self, "x3_min_population", None))

    def _conv(self, conv, x, y, h, w, oh, ow, acc=False, x2=None, bn=None, training=True):
        """'same' (stride 1) or unpadded strided conv of x [B,h,w,cin] into y [B,oh,ow,cout];
        with `bn`, also that BN's statistics of y (fused into the conv epilogue in training)."""
        k, s = conv.k, conv.stride
        if s == 1:
            pt, pl = (k - 1) // 2, (k - 1) // 2
        else:
            pt = pl = 0
        args = K.conv_args(x, x2, k, k, s, pt, pl, oh, ow, conv.cout,
                           math=self._math(conv, oh, ow))
        if bn is not None:
            assert not acc and x2 is None
            bn.conv_fwd_stats(args, conv.w_nat, conv.b, y, self.B * oh * ow, training)
        else:
            K.conv2d_fwd(args, conv.w_nat, conv.b, y, accumulate=acc)
        return args

    def forward(self, training=True, step=0, image_offset=0):
        A, B = self.act, self.B
        H, W = self.H, self.W
        h, w = H // 2, W // 2
        # stem: ZeroPadding2D(3) + 7x7/2 valid conv (+bias), BN, ReLU, ZeroPadding2D(1) + pool
        x0, w0 = A["input"], self.stem.w_nat
        args = K.conv_args(x0, None, 7, 7, 2, 3, 3, h, w, 64, math=self._math(self.stem, h, w))
        self.stem_bn.conv_fwd_stats(args, w0, self.stem.b, A["conv1_pre"], B * h * w, training)
        self.stem_bn.apply(A["conv1_pre"], B * h * w, "relu", A["conv1_relu"], training)
        K.maxpool2d_fwd(A["conv1_relu"], 3, 2, 1, 1, A["pool1_pool"], self.pool_argmax)
        x = A["pool1_pool"]
        forked = {}
        for blk in self.blocks:
            x = self._block_fwd(blk, x, training)
            if self.overlap_ffl:
                for d in self.ffls:
                    if d["tap"] == blk["name"] + "out":
                        forked[d["name"]] = self._fork_left(d, training)
        h, w = x.shape[1], x.shape[2]
        K.upsample2x_fwd(A["conv5_block3_out"], A["conv5_up"])
        up = A["conv5_up"]
        for d in self.ffls:
            up = self._ffl_fwd(d, A[d["tap"]], up, training, forked.get(d["name"]))
        h, w = up.shape[1], up.shape[2]
        rows = B * h * w
        self._conv(self.aol0, up, A["aol/pre0"], h, w, h, w, bn=self.aol_bn, training=training)
        self.aol_bn.apply(A["aol/pre0"], rows, "relu", A["aol/act0"], training)
        self._conv(self.aol1, A["aol/act0"], A["aol/pre1"], h, w, h, w)
        K.upsample2x_fwd(A["aol/pre1"], A["aol/up"])
        self._conv(self.aol2, A["aol/up"], A["pred"], H, W, H, W)
        return A["pred"]

    def _block_fwd(self, blk, x, training):
        A, B, n = self.act, self.B, blk["name"]
        h, w, oh, ow = blk["hw"]
        rows = B * oh * ow
        join = None
        if blk["proj"]:
            def shortcut():
                self._conv(blk["c0"], x, A[n + "0_pre"], h, w, oh, ow,
                           bn=blk["bn0"], training=training)
                blk["bn0"].apply(A[n + "0_pre"], rows, "none", A[n + "0_bn"], training)
            if self.overlap_proj:
                # the projection shortcut beside conv1 -> conv2 -> conv3 (joined at the add)
                stream, fork, join = self._proj_side()
                fork.record(torch.cuda.current_stream(self.device))
                with torch.cuda.stream(stream), K.workspace_scope("/proj_side"):
                    stream.wait_event(fork)
                    shortcut()
                    join.record(stream)
            else:
                shortcut()
            sc = A[n + "0_bn"]
        else:
            sc = x
        self._conv(blk["c1"], x, A[n + "1_pre"], h, w, oh, ow, bn=blk["bn1"], training=training)
        blk["bn1"].apply(A[n + "1_pre"], rows, "relu", A[n + "1_relu"], training)
        self._conv(blk["c2"], A[n + "1_relu"], A[n + "2_pre"], oh, ow, oh, ow, bn=blk["bn2"],
                   training=training)
        blk["bn2"].apply(A[n + "2_pre"], rows, "relu", A[n + "2_relu"], training)
        self._conv(blk["c3"], A[n + "2_relu"], A[n + "3_pre"], oh, ow, oh, ow, bn=blk["bn3"],
                   training=training)
        if join is not None:
            torch.cuda.current_stream(self.device).wait_event(join)
        blk["bn3"].add_apply(A[n + "3_pre"], rows, sc, "relu", A[n + "out"], training)
        return A[n + "out"]

    def _proj_side(self):
        """(stream, fork, join) of the projection-shortcut branch (one branch in flight at a time:
        each is joined inside its block)."""
        if not hasattr(self, "_pside"):
            self._pside = (torch.cuda.Stream(device=self.device), torch.cuda.Event(),
                           torch.cuda.Event())
        return self._pside

    def _bottleneck_fwd(self, bt, x, h, w, training):
        A, n = self.act, bt["name"]
        rows = self.B * h * w
        for half in (0, 3):
            c, b = bt["convs"], bt["bns"]
            self._conv(c[half], x, A[f"{n}/pre{half}"], h, w, h, w, bn=b[half], training=training)
            b[half].apply(A[f"{n}/pre{half}"], rows, "relu", A[f"{n}/act{half}"], training)
            self._conv(c[half + 1], A[f"{n}/act{half}"], A[f"{n}/pre{half + 1}"], h, w, h, w,
                       bn=b[half + 1], training=training)
            b[half + 1].apply(A[f"{n}/pre{half + 1}"], rows, "relu", A[f"{n}/act{half + 1}"],
                              training)
            self._conv(c[half + 2], A[f"{n}/act{half + 1}"], A[f"{n}/pre{half + 2}"], h, w, h, w,
                       bn=b[half + 2], training=training)
            b[half + 2].add_apply(A[f"{n}/pre{half + 2}"], rows, x, "relu", A[f"{n}/out{half}"],
                                  training)
            x = A[f"{n}/out{half}"]
        return x

    def _ffl_left_fwd(self, d, left, training):
        A, n = self.act, d["name"]
        h, w = d["hw"]
        self._conv(d["conv0"], left, A[n + "/left_pre"], h, w, h, w,
                   bn=d["bn0"], training=training)
        d["bn0"].apply(A[n + "/left_pre"], self.B * h * w, "none", A[n + "/left_bn"], training)
        return self._bottleneck_fwd(d["left"], A[n + "/left_bn"], h, w, training)

    def _ffl_side(self):
        """(stream, {ffl name [+ "/bwd"]: (fork, join) events}) of the FFL left branches."""
        if not hasattr(self, "_fside"):
            evs = {}
            for f in self.ffls:
                for k in (f["name"], f["name"] + "/bwd"):
                    evs[k] = (torch.cuda.Event(), torch.cuda.Event())
            self._fside = (torch.cuda.Stream(device=self.device), evs)
        return self._fside

    def _fork_left(self, d, training):
        """Run d's left branch on the FFL side stream once the main stream has produced its tap;
        returns (left-branch output, join event). The side stream's calls use their own
        workspaces (kernels.workspace_scope); every tensor they write belongs to the branch."""
        stream, evs = self._ffl_side()
        fork, join = evs[d["name"]]
        fork.record(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(stream), K.workspace_scope("/ffl_side"):
            stream.wait_event(fork)
            xl = self._ffl_left_fwd(d, self.act[d["tap"]], training)
            join.record(stream)
        return xl, join

    def _ffl_fwd(self, d, left, up, training, forked=None):
        A, n = self.act, d["name"]
        h, w = d["hw"]
        rows = self.B * h * w
        if forked is None:
            xl = self._ffl_left_fwd(d, left, training)
        else:
            xl, join = forked
        self._conv(d["conv1"], up, A[n + "/up_pre"], h, w, h, w, bn=d["bn1"], training=training)
        if forked is not None:
            torch.cuda.current_stream(self.device).wait_event(join)
        d["bn1"].add_apply(A[n + "/up_pre"], rows, xl, "none", A[n + "/sum"], training)
        xd = self._bottleneck_fwd(d["down"], A[n + "/sum"], h, w, training)
        K.upsample2x_fwd(xd, A[n + "/out"])
        return A[n + "/out"]

    # ------------------------------------------------------------------ backward
    def _wslot(self, conv, slot=0):
        """Buffer slot of a trainable conv's output gradient: its own while the side stream may
        still read it (weight-gradient overlap), else the shared per-shape slot."""
        return ("w", conv.name) if self._side else slot

    def _wgrad_side(self):
        """(stream, per-conv fork events) of the decoder's weight-gradient side stream."""
        if not hasattr(self, "_wside"):
            self._wside = (torch.cuda.Stream(device=self.device),
                           {c.name: torch.cuda.Event() for c in self.convs if c.trainable})
        return self._wside

    def _wgrad_dgrad(self, conv, x, gy, h, w, oh, ow, gx, gx_acc=False):
        """dW (+db) for trainable convs, dX (=|+=) into gx when gx is given. With the weight-
        gradient overlap, dW and db run on the side stream, forked here (gy complete)."""
        k, s = conv.k, conv.stride
        pt = pl = ((k - 1) // 2 if s == 1 else 0)
        args = K.conv_args(x, None, k, k, s, pt, pl, oh, ow, conv.cout,
                           math=self._math(conv, oh, ow, bwd=True))
        if conv.trainable:
            if self._side and not self._in_fside:
                def wg(args=args, gy=gy, rows=self.B * oh * ow, conv=conv):
                    K.conv2d_wgrad(args, gy, conv.dw)
                    if conv.db is not None:
                        K.channel_sum(gy, rows, conv.cout, conv.db, ws_key="reduce_side")
                if self.overlap_wgrad == 2:
                    self._deferred.append(wg)
                else:
                    wstream, fork = self._wgrad_side()
                    fork[conv.name].record(torch.cuda.current_stream(self.device))
                    with torch.cuda.stream(wstream):
                        wstream.wait_event(fork[conv.name])
                        wg()
            else:  # single stream, or on the FFL side stream (already beside the main chain)
                K.conv2d_wgrad(args, gy, conv.dw)
                if conv.db is not None:
                    K.channel_sum(gy, self.B * oh * ow, conv.cout, conv.db)
        if gx is not None:
            K.conv2d_dgrad(args, gy, conv.w_dg, gx, None, acc1=gx_acc)

    def param_offset(self, name):
        """Offset of a trainable tensor in the flat params / grads buffers."""
        return next(off for n, _, off in self.params.specs if n == name)

    def backward(self, dpred):
        """Backward from d loss / d pred: fills self.grads (decoder kernels/biases, BN params)."""
        A, G, B = self.act, self.gact, self.B
        # decoder weight gradients on a side stream (EffNetFF.backward)
        self._side = bool(self.overlap_wgrad)
        self._deferred = []
        main = torch.cuda.current_stream(self.device)
        H, W = self.H, self.W
        h, w = H // 2, W // 2
        # AdaptiveOutputLayer
        self._wgrad_dgrad(self.aol2, A["aol/up"], dpred, H, W, H, W, G["aol/up"])
        K.upsample2x_bwd(G["aol/up"], G["aol/pre1"])
        self._wgrad_dgrad(self.aol1, A["aol/act0"], G["aol/pre1"], h, w, h, w, G["aol/act0"])
        g0 = self._gpre_buf(A["aol/pre0"].shape, self._wslot(self.aol0))
        self.aol_bn.bwd(A["aol/pre0"], G["aol/act0"], B * h * w, "relu", g0)
        self._wgrad_dgrad(self.aol0, A["ffl2/out"], g0, h, w, h, w, G["ffl2/out"])
        # feature fusion layers, top (ffl2) to bottom (ffl0)
        # (with the weight-gradient overlap, each FFL's left branch runs on the FFL side stream
        # from the moment its input gradient exists; the encoder joins it at the tap)
        tap_join = {}
        for i in range(len(self.ffls) - 1, -1, -1):
            d = self.ffls[i]
            up = A["conv5_up"] if i == 0 else A[self.ffls[i - 1]["name"] + "/out"]
            gup = G["conv5_up"] if i == 0 else G[self.ffls[i - 1]["name"] + "/out"]
            j = self._ffl_bwd(d, A[d["tap"]], G[d["tap"]], up, gup,
                              fork=self._side and bool(self.overlap_ffl))
            if j is not None:
                tap_join[d["tap"]] = j
        if self._side and self._deferred:  # overlap mode 2: beside the encoder backward
            wstream, fork = self._wgrad_side()
            ev = fork[self.aol0.name]
            ev.record(main)
            with torch.cuda.stream(wstream):
                wstream.wait_event(ev)
                for wg in self._deferred:
                    wg()
        self._deferred = []
        K.upsample2x_bwd(G["conv5_up"], G["conv5_block3_out"])
        # encoder (taps already hold their decoder gradient: accumulate onto them)
        for bi in range(len(self.blocks) - 1, -1, -1):
            blk = self.blocks[bi]
            if bi == 0:
                xn = "pool1_pool"
            else:
                xn = self.blocks[bi - 1]["name"] + "out"
            if xn in tap_join:  # this block accumulates onto the tap's decoder gradient
                main.wait_event(tap_join.pop(xn))
            self._block_bwd(blk, A[xn], G[xn], xn in TAPS)
        hp, wp = A["pool1_pool"].shape[1:3]
        K.maxpool2d_bwd(G["pool1_pool"], self.pool_argmax, 3, 2, 1, 1, G["conv1_relu"])
        self.stem_bn.bwd(A["conv1_pre"], G["conv1_relu"], B * h * w, "relu", None)
        for j in tap_join.values():  # (none left: every tap feeds an encoder block)
            main.wait_event(j)
        if self._side:  # join: every weight gradient is final on the caller's stream
            main.wait_stream(self._wgrad_side()[0])
        self._side = False

    def _block_bwd(self, blk, x, gx, gx_is_tap):
        A, G, B, n = self.act, self.gact, self.B, blk["name"]
        h, w, oh, ow = blk["hw"]
        rows = B * oh * ow
        gout = G[n + "out"]
        g3 = self._gpre_buf(A[n + "3_pre"].shape)
        join = None
        if blk["proj"]:
            gsc = G[n + "0_bn"]
            blk["bn3"].add_bwd(A[n + "3_pre"], gout, rows, A[n + "0_bn"], "relu", g3, gsc)

            def shortcut():  # bn0 backward + conv0 dX into gx (slot 2: g3 has 0_pre's shape)
                g0 = self._gpre_buf(A[n + "0_pre"].shape, 2)
                blk["bn0"].bwd(A[n + "0_pre"], gsc, rows, "none", g0)
                self._wgrad_dgrad(blk["c0"], x, g0, h, w, oh, ow, gx, gx_acc=gx_is_tap)
            if self.overlap_proj:  # beside conv3 -> conv2 -> conv1's backward
                stream, fork, join = self._proj_side()
                fork.record(torch.cuda.current_stream(self.device))
                with torch.cuda.stream(stream), K.workspace_scope("/proj_side"):
                    stream.wait_event(fork)
                    shortcut()
                    join.record(stream)
            else:
                shortcut()
        else:
            blk["bn3"].add_bwd(A[n + "3_pre"], gout, rows, x, "relu", g3, gx,
                               dres_acc=gx_is_tap)
        self._wgrad_dgrad(blk["c3"], A[n + "2_relu"], g3, oh, ow, oh, ow, G[n + "2_relu"])
        g2 = self._gpre_buf(A[n + "2_pre"].shape, 1)
        blk["bn2"].bwd(A[n + "2_pre"], G[n + "2_relu"], rows, "relu", g2)
        self._wgrad_dgrad(blk["c2"], A[n + "1_relu"], g2, oh, ow, oh, ow, G[n + "1_relu"])
        g1 = self._gpre_buf(A[n + "1_pre"].shape, 1)
        blk["bn1"].bwd(A[n + "1_pre"], G[n + "1_relu"], rows, "relu", g1)
        if join is not None:  # the shortcut's dX is in gx: conv1's dX accumulates onto it
            torch.cuda.current_stream(self.device).wait_event(join)
        self._wgrad_dgrad(blk["c1"], x, g1, h, w, oh, ow, gx, gx_acc=True)

    def _bottleneck_bwd(self, bt, x, gx, gy, h, w):
        """gy: gradient of the bottleneck output; writes the input gradient into gx."""
        A, G, n = self.act, self.gact, bt["name"]
        rows = self.B * h * w
        c, b = bt["convs"], bt["bns"]
        for half in (3, 0):
            xin = x if half == 0 else A[f"{n}/out0"]
            gin = gx if half == 0 else G[f"{n}/out0"]
            gp = self._gpre_buf(A[f"{n}/pre{half + 2}"].shape, self._wslot(c[half + 2]))
            b[half + 2].add_bwd(A[f"{n}/pre{half + 2}"], gy, rows, xin, "relu", gp, gin)
            self._wgrad_dgrad(c[half + 2], A[f"{n}/act{half + 1}"], gp, h, w, h, w,
                              G[f"{n}/act{half + 1}"])
            gq = self._gpre_buf(A[f"{n}/pre{half + 1}"].shape, self._wslot(c[half + 1]))
            b[half + 1].bwd(A[f"{n}/pre{half + 1}"], G[f"{n}/act{half + 1}"], rows, "relu", gq)
            self._wgrad_dgrad(c[half + 1], A[f"{n}/act{half}"], gq, h, w, h, w,
                              G[f"{n}/act{half}"])
            gq0 = self._gpre_buf(A[f"{n}/pre{half}"].shape, self._wslot(c[half], 1))
            b[half].bwd(A[f"{n}/pre{half}"], G[f"{n}/act{half}"], rows, "relu", gq0)
            self._wgrad_dgrad(c[half], xin, gq0, h, w, h, w, gin, gx_acc=True)
            gy = gin

    def _ffl_left_bwd(self, d, left, gleft):
        A, G, n = self.act, self.gact, d["name"]
        h, w = d["hw"]
        # block_left receives G[sum] unchanged (identity branch of the add)
        self._bottleneck_bwd(d["left"], A[n + "/left_bn"], G[n + "/left_bn"], G[n + "/sum"],
                             h, w)
        gl = self._gpre_buf(A[n + "/left_pre"].shape, self._wslot(d["conv0"]))
        d["bn0"].bwd(A[n + "/left_pre"], G[n + "/left_bn"], self.B * h * w, "none", gl)
        self._wgrad_dgrad(d["conv0"], left, gl, h, w, h, w, gleft)

    def _ffl_bwd(self, d, left, gleft, up, gup, fork=False):
        """Backward of one feature-fusion layer. fork: the left branch (which needs only G[sum]
        and writes only its own buffers, its weight gradients and the tap's gradient) runs on the
        FFL side stream, its dW inline there; returns its join event (else None)."""
        A, G, n = self.act, self.gact, d["name"]
        h, w = d["hw"]
        rows = self.B * h * w
        gd = G[d["down"]["name"] + "/out3"]
        K.upsample2x_bwd(G[n + "/out"], gd)
        # block_down: input gradient lands in G[sum]; sum = bn1(up_pre) + block_left output
        self._bottleneck_bwd(d["down"], A[n + "/sum"], G[n + "/sum"], gd, h, w)
        join = None
        if fork:
            stream, evs = self._ffl_side()
            fk, join = evs[n + "/bwd"]
            fk.record(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(stream), K.workspace_scope("/ffl_side"):
                stream.wait_event(fk)
                self._in_fside = True
                try:
                    self._ffl_left_bwd(d, left, gleft)
                finally:
                    self._in_fside = False
                join.record(stream)
        gu = self._gpre_buf(A[n + "/up_pre"].shape, self._wslot(d["conv1"]))
        d["bn1"].bwd(A[n + "/up_pre"], G[n + "/sum"], rows, "none", gu)
        self._wgrad_dgrad(d["conv1"], up, gu, h, w, h, w, gup)
        if not fork:
            self._ffl_left_bwd(d, left, gleft)
        return join

    # ------------------------------------------------------------------ optimizer / counts
    def adam_state(self):
        if not hasattr(self, "_adam"):
            self._adam = [torch.zeros_like(self.params.buf) for _ in range(3)]
        return self._adam

    def adam_step(self, lr, step, grad_scale=1.0, beta1=0.9, beta2=0.999, eps=1e-7):
        m, v, vh = self.adam_state()
        K.adam_amsgrad(self.params.buf, self.grads.buf, m, v, vh, lr, step, beta1, beta2, eps,
                       grad_scale)
        self.refresh_trainable()

    def count_trainable(self):
        return sum(int(np.prod(s)) for _, s, _ in self.params.specs)

    def conv_flops_per_image(self):
        """Algorithmic dense-conv FLOPs per image of one train step (fwd + encoder dX except the
        stem, decoder fwd + dX + dW): 142.54 GFLOP at 448x448."""
        H, W = self.H, self.W
        f = (H // 2) * (W // 2) * 49 * 3 * 64
        for blk in self.blocks:
            h, w, oh, ow = blk["hw"]
            cin, fl = blk["cin"], blk["f"]
            if blk["proj"]:
                f += 2 * oh * ow * cin * 4 * fl
            f += 2 * oh * ow * (cin * fl + 9 * fl * fl + fl * 4 * fl)
        dec = 0
        for d in self.ffls:
            h, w = d["hw"]
            dec += h * w * 9 * (d["conv0"].cin + d["conv1"].cin) * d["inter"]
            for bt in (d["left"], d["down"]):
                p, q = bt["p"], bt["q"]
                dec += 2 * h * w * (p * q + 9 * q * q + q * p)
        dec += (H // 2) * (W // 2) * (9 * 64 * 64 + 9 * 64) + H * W
        return 2.0 * (f + 3 * dec)
