"""torch-CPU (fp64) restatement of the ff_effnet graph — TEST INFRASTRUCTURE (see oracle/__init__).

Restates ``EffNetFullyFledged.get_model_and_normalization`` (pldepth/models/pl_hourglass.py:45-100)
with the semantics of its third-party pieces (TF/Keras 2.3-2.8, not vendored, PARITY UNPINNED —
no TF here; restated from the published keras.applications.efficientnet / Keras layer sources):

  * Rescaling(1/255) -> Normalization((x - mean) / max(sqrt(var), 1e-7))
  * stem: ZeroPadding2D(correct_pad) -> Conv2D(32, 3, s2, valid, no bias) -> BN -> swish
  * 16 MBConv blocks (B0 table): [expand 1x1 -> BN -> swish] -> [ZeroPadding2D(correct_pad) if
    s2] DepthwiseConv2D(k, s, 'same'|'valid') -> BN -> swish -> SE(GAP -> 1x1 swish -> 1x1
    sigmoid -> multiply) -> project 1x1 -> BN -> [Dropout(noise (N,1,1,1)) + residual]
  * top 1x1 -> 1280 -> BN -> swish
  * decoder (pl_hourglass.py:59-96): 5 x [Conv2D 3x3 'same' + bias -> BN -> ReLU ->
    UpSampling2D(bilinear, half-pixel)] with Concatenate([x, skip]) after stages 1-3
    (skips: block6a/block4a/block3a _expand_activation), final Conv2D(1, 3x3) + bias.
  * BatchNormalization training mode: batch mean / biased variance, epsilon 1e-3.

Layout: NCHW inside, NHWC at the boundary; weights are a dict keyed by Keras layer names with
Keras layouts (Conv2D kernel HWIO, DepthwiseConv2D kernel [k][k][c][1] stored as [k][k][c]).
"""
import torch
import torch.nn.functional as F

BN_EPS = 1e-3

# keras.applications.efficientnet DEFAULT_BLOCKS_ARGS (B0: width = depth = 1.0)
B0_BLOCKS = [
    # kernel, repeats, filters_in, filters_out, expand_ratio, strides
    (3, 1, 32, 16, 1, 1),
    (3, 2, 16, 24, 6, 2),
    (5, 2, 24, 40, 6, 2),
    (3, 3, 40, 80, 6, 2),
    (5, 3, 80, 112, 6, 1),
    (5, 4, 112, 192, 6, 2),
    (3, 1, 192, 320, 6, 1),
]
SE_RATIO = 0.25
DROP_CONNECT = 0.2
DECODER = [  # (name, cout, skip tap after upsampling or None)
    ("dec_conv0", 672, "block6a_expand_activation"),
    ("dec_conv1", 240, "block4a_expand_activation"),
    ("dec_conv2", 144, "block3a_expand_activation"),
    ("dec_conv3", 32, None),
    ("dec_conv4", 32, None),
]


def block_specs():
    """Expanded per-block list: (name, k, s, cin, cout, expand, drop_rate)."""
    out = []
    total = sum(r for _, r, *_ in B0_BLOCKS)
    b = 0
    for i, (k, reps, fin, fout, ex, s) in enumerate(B0_BLOCKS):
        for j in range(reps):
            cin = fin if j == 0 else fout
            st = s if j == 0 else 1
            out.append((f"block{i + 1}{chr(97 + j)}_", k, st, cin, fout, ex,
                        DROP_CONNECT * b / total))
            b += 1
    return out


def correct_pad(size, k):
    """imagenet_utils.correct_pad for an even/odd spatial size: (before, after)."""
    adjust = 1 - size % 2
    c = k // 2
    return c - adjust, c


def same_pad(size, k, s):
    out = -(-size // s)
    total = max((out - 1) * s + k - size, 0)
    return total // 2, total - total // 2, out


def conv(x, w_hwio, bias=None, stride=1, pads=None):
    """x NCHW; w HWIO; pads = (top, bottom, left, right) explicit zero padding."""
    if pads is not None:
        t, b, l, r = pads
        x = F.pad(x, (l, r, t, b))
    w = w_hwio.permute(3, 2, 0, 1).contiguous()
    return F.conv2d(x, w, bias, stride=stride)


def conv_same(x, w_hwio, bias=None, stride=1):
    k = w_hwio.shape[0]
    t, b, _ = same_pad(x.shape[2], k, stride)
    l, r, _ = same_pad(x.shape[3], w_hwio.shape[1], stride)
    return conv(x, w_hwio, bias, stride, (t, b, l, r))


def dwconv(x, w_kkc, stride, pads):
    t, b, l, r = pads
    x = F.pad(x, (l, r, t, b))
    c = x.shape[1]
    w = w_kkc.permute(2, 0, 1).unsqueeze(1).contiguous()  # [c,1,k,k]
    return F.conv2d(x, w, None, stride=stride, groups=c)


def bn_train(x, gamma, beta, eps=BN_EPS):
    mean = x.mean(dim=(0, 2, 3), keepdim=True)
    var = ((x - mean) ** 2).mean(dim=(0, 2, 3), keepdim=True)
    xh = (x - mean) / torch.sqrt(var + eps)
    return xh * gamma.view(1, -1, 1, 1) + beta.view(1, -1, 1, 1)


def swish(x):
    return x * torch.sigmoid(x)


def up2(x):
    return F.interpolate(x, scale_factor=2, mode="bilinear", align_corners=False)


def bn_infer(x, gamma, beta, mmean, mvar, eps=BN_EPS):
    """Keras BatchNormalization(training=False): the moving statistics."""
    v = lambda t: t.view(1, -1, 1, 1)
    return (x - v(mmean)) / torch.sqrt(v(mvar) + eps) * v(gamma) + v(beta)


_TRAINING = [True]
_STATS = [None]  # forward(bn_stats=...): {bn name: (batch mean, biased batch variance)}


def _bn(P, name, x):
    if _TRAINING[0]:
        if _STATS[0] is not None:
            m = x.mean(dim=(0, 2, 3))
            _STATS[0][name] = (m, ((x - m.view(1, -1, 1, 1)) ** 2).mean(dim=(0, 2, 3)))
        return bn_train(x, P[name + "/gamma"], P[name + "/beta"])
    return bn_infer(x, P[name + "/gamma"], P[name + "/beta"], P[name + "/moving_mean"],
                    P[name + "/moving_variance"])


def forward(P, x_nhwc, drop_scales=None, taps=None, training=True, bn_stats=None,
            relu_masks=None):
    """ff_effnet forward. P: dict of fp64 tensors (Keras names/layouts). x_nhwc: [N,H,W,3] in
    [0,1]. drop_scales: {block_name: [N] keep/(1-rate) factors} (None = drop-connect off).
    taps: optional dict receiving intermediate NHWC activations. training=False: every BN on
    its moving statistics (Keras predict / validation; drop-connect is then off). bn_stats:
    optional dict receiving every training-mode BN's batch mean and variance. relu_masks:
    optional {decoder stage: [N,C,H,W] 0/1} replacing that stage's ReLU by a multiplication
    with the given mask (the same piecewise-linear branch as another implementation took, for
    comparing arithmetic where a pre-activation lies within rounding of 0). Returns
    [N,H,W,1]."""
    if bn_stats is not None:
        _STATS[0] = bn_stats
        try:
            return forward(P, x_nhwc, drop_scales, taps, training, relu_masks=relu_masks)
        finally:
            _STATS[0] = None
    if not training:
        _TRAINING[0] = False
        try:
            return forward(P, x_nhwc, None, taps, True, relu_masks=relu_masks)
        finally:
            _TRAINING[0] = True
    acts = taps if taps is not None else {}
    x = x_nhwc.permute(0, 3, 1, 2)
    mean = P["normalization/mean"].view(1, 3, 1, 1)
    var = P["normalization/variance"].view(1, 3, 1, 1)
    x = (x / 255.0 - mean) / torch.clamp(torch.sqrt(var), min=1e-7)
    t, b = correct_pad(x.shape[2], 3)
    l, r = correct_pad(x.shape[3], 3)
    x = conv(x, P["stem_conv/kernel"], None, 2, (t, b, l, r))
    x = swish(_bn(P, "stem_bn", x))
    acts["stem_activation"] = x
    for name, k, s, cin, cout, ex, rate in block_specs():
        inp = x
        if ex != 1:
            x = conv(x, P[name + "expand_conv/kernel"])
            x = swish(_bn(P, name + "expand_bn", x))
            acts[name + "expand_activation"] = x
        if s == 2:
            t, b = correct_pad(x.shape[2], k)
            l, r = correct_pad(x.shape[3], k)
        else:
            t, b, _ = same_pad(x.shape[2], k, 1)
            l, r, _ = same_pad(x.shape[3], k, 1)
        x = dwconv(x, P[name + "dwconv/depthwise_kernel"], s, (t, b, l, r))
        x = swish(_bn(P, name + "bn", x))
        se = x.mean(dim=(2, 3), keepdim=True)
        se = swish(conv(se, P[name + "se_reduce/kernel"], P[name + "se_reduce/bias"]))
        se = torch.sigmoid(conv(se, P[name + "se_expand/kernel"], P[name + "se_expand/bias"]))
        x = x * se
        x = conv(x, P[name + "project_conv/kernel"])
        x = _bn(P, name + "project_bn", x)
        if s == 1 and cin == cout:
            if drop_scales is not None and name in drop_scales:
                x = x * drop_scales[name].view(-1, 1, 1, 1)
            x = x + inp
        acts[name + "output"] = x
    x = conv(x, P["top_conv/kernel"])
    x = swish(_bn(P, "top_bn", x))
    acts["top_activation"] = x
    for i, (name, cout, skip) in enumerate(DECODER):
        x = conv_same(x, P[name + "/kernel"], P[name + "/bias"])
        z = _bn(P, f"dec_bn{i}", x)
        acts[f"dec{i}_z"] = z  # the pre-activation (its sign decides the ReLU branch)
        if relu_masks is not None and i in relu_masks:
            x = z * relu_masks[i].to(z.dtype)
        else:
            x = torch.relu(z)
        x = up2(x)
        if skip is not None:
            x = torch.cat([x, acts[skip]], dim=1)
        acts[f"dec{i}"] = x
    x = conv_same(x, P["dec_conv5/kernel"], P["dec_conv5/bias"])
    out = x.permute(0, 2, 3, 1)
    return out


def trainable_names(P):
    """Names the reference trains: decoder conv kernels/biases, every BN gamma/beta."""
    return [k for k in P if k.startswith("dec_conv") or k.endswith("/gamma") or k.endswith("/beta")]


def train_step_grads(P, x_nhwc, dloss_dpred, drop_scales=None, relu_masks=None):
    """Gradients of the trainable parameters for an upstream gradient dloss/dpred (fp64);
    relu_masks as in forward."""
    Q = {k: (v.detach().clone().requires_grad_(True) if k in set(trainable_names(P))
             else v.detach()) for k, v in P.items()}
    out = forward(Q, x_nhwc, drop_scales, relu_masks=relu_masks)
    out.backward(dloss_dpred)
    return {k: Q[k].grad.detach() for k in trainable_names(P)}, out.detach()
