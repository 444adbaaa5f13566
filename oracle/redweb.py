"""torch-CPU (fp64) restatement of the ff_redweb graph — TEST INFRASTRUCTURE (see oracle/__init__).

Restates ``ReDWebNetTFVersion.get_model_and_normalization`` (pldepth/models/redweb.py:402-434)
and the third-party ResNet50 it builds on (keras.applications.resnet, TF 2.3-2.8, not vendored,
PARITY UNPINNED — no TF here; restated from the published Keras sources):

  encoder (redweb.py:410, include_top=False; every Conv2D has a bias, BN epsilon 1.001e-5):
    conv1_pad ZeroPadding2D(3) -> conv1_conv 7x7/2 (64) -> conv1_bn -> relu ->
    pool1_pad ZeroPadding2D(1) -> pool1_pool MaxPooling2D(3, 2)
    conv{2,3,4,5} = stack1(filters 64/128/256/512, blocks 3/4/6/3, stride1 1/2/2/2):
      block1(x, f, stride, conv_shortcut) (Keras resnet.block1):
        shortcut = BN(Conv1x1/stride(4f)(x)) for the first block of a stack, else x
        x = relu(BN(Conv1x1/stride(f)(x))); x = relu(BN(Conv3x3 'same'(f)(x)))
        x = BN(Conv1x1(4f)(x)); out = relu(shortcut + x)
  taps (redweb.py:418-421): conv2_block3_out, conv3_block4_out, conv4_block3_out,
  conv5_block3_out (note: conv4_block3, not the stack's last block 6)
  decoder (redweb.py:423-428):
    up(conv5_block3_out) -> FeatureFusionLayer(256,256)([conv4_block3_out, .])
    -> FFL(128,128)([conv3_block4_out, .]) -> FFL(64,64)([conv2_block3_out, .])
    -> AdaptiveOutputLayer
    FFL (redweb.py:225-290): left = block_left(BN(conv3x3(in_left)));  up = BN(conv3x3(in_up));
      x = up2(block_down(left + up)); convs without bias, Keras BN (epsilon 1e-3)
    BottleneckConvLayer(p) (redweb.py:67-165): two residual bottlenecks 1x1(p/4)-3x3(p/4)-1x1(p)
      with BN after each conv, relu between, `out += residual; relu`
    AdaptiveOutputLayer (redweb.py:293-338): conv3x3(64)+bias -> BN -> relu -> conv3x3(1)+bias
      -> up2 -> conv1x1(1)+bias (the LeakyReLU it builds is never called)
  preprocess_input (caffe): RGB->BGR, minus [103.939, 116.779, 123.68], applied to the [0,1]
  images by the data pipeline (PLDepth.py:169-173), not inside the model.

Weight names: Keras ResNet50 layer names for the encoder (conv2_block1_0_conv/kernel, ...);
the decoder's subclassed layers are named ffl{0,1,2}/{conv0,bn0,conv1,bn1},
ffl{i}/{block_left,block_down}/{conv0..conv5,bn0..bn5}, aol/{conv0,bn0,conv1,conv2}.
"""
import torch
import torch.nn.functional as F

from .effnet import conv, conv_same, up2

RESNET_BN_EPS = 1.001e-5
DEC_BN_EPS = 1e-3
CAFFE_MEAN_BGR = (103.939, 116.779, 123.68)
# keras.applications.resnet.ResNet50 stack_fn: (name, filters, blocks, stride1)
RESNET50_STACKS = [("conv2", 64, 3, 1), ("conv3", 128, 4, 2), ("conv4", 256, 6, 2),
                   ("conv5", 512, 3, 2)]
TAPS = ("conv2_block3_out", "conv3_block4_out", "conv4_block3_out", "conv5_block3_out")
# (name, inter_planes, out_planes, left tap, left channels, up channels)
FFLS = [("ffl0", 256, 256, "conv4_block3_out", 1024, 2048),
        ("ffl1", 128, 128, "conv3_block4_out", 512, 256),
        ("ffl2", 64, 64, "conv2_block3_out", 256, 128)]


def param_specs():
    """[(name, shape, kind)] with kind in {'frozen', 'trainable', 'stat'} for every tensor of
    the model (Keras layouts: Conv2D kernel HWIO)."""
    out = []

    def conv_(name, k, cin, cout, bias, trainable):
        kind = "trainable" if trainable else "frozen"
        out.append((name + "/kernel", (k, k, cin, cout), kind))
        if bias:
            out.append((name + "/bias", (cout,), kind))

    def bn_(name, c):
        out.append((name + "/gamma", (c,), "trainable"))
        out.append((name + "/beta", (c,), "trainable"))
        out.append((name + "/moving_mean", (c,), "stat"))
        out.append((name + "/moving_variance", (c,), "stat"))

    conv_("conv1_conv", 7, 3, 64, True, False)
    bn_("conv1_bn", 64)
    cin = 64
    for name, f, blocks, _ in RESNET50_STACKS:
        for b in range(1, blocks + 1):
            pre = f"{name}_block{b}_"
            if b == 1:
                conv_(pre + "0_conv", 1, cin, 4 * f, True, False)
                bn_(pre + "0_bn", 4 * f)
            conv_(pre + "1_conv", 1, cin, f, True, False)
            bn_(pre + "1_bn", f)
            conv_(pre + "2_conv", 3, f, f, True, False)
            bn_(pre + "2_bn", f)
            conv_(pre + "3_conv", 1, f, 4 * f, True, False)
            bn_(pre + "3_bn", 4 * f)
            cin = 4 * f

    def bottleneck_(name, p):
        q = p // 4
        for i, (k, ci, co) in enumerate([(1, p, q), (3, q, q), (1, q, p)] * 2):
            conv_(f"{name}/conv{i}", k, ci, co, False, True)
            bn_(f"{name}/bn{i}", co)

    for name, inter, outp, _, cl, cu in FFLS:
        conv_(name + "/conv0", 3, cl, inter, False, True)
        bn_(name + "/bn0", inter)
        conv_(name + "/conv1", 3, cu, inter, False, True)
        bn_(name + "/bn1", inter)
        bottleneck_(name + "/block_left", inter)
        bottleneck_(name + "/block_down", outp)
    conv_("aol/conv0", 3, 64, 64, True, True)
    bn_("aol/bn0", 64)
    conv_("aol/conv1", 3, 64, 1, True, True)
    conv_("aol/conv2", 1, 1, 1, True, True)
    return out


def bn_train(x, gamma, beta, eps):
    mean = x.mean(dim=(0, 2, 3), keepdim=True)
    var = ((x - mean) ** 2).mean(dim=(0, 2, 3), keepdim=True)
    xh = (x - mean) / torch.sqrt(var + eps)
    return xh * gamma.view(1, -1, 1, 1) + beta.view(1, -1, 1, 1)


def _bn(P, name, x, eps):
    return bn_train(x, P[name + "/gamma"], P[name + "/beta"], eps)


def caffe_preprocess(x_nhwc):
    """keras resnet preprocess_input (mode 'caffe') on [0,1] RGB: BGR, minus the ImageNet mean."""
    x = x_nhwc[..., [2, 1, 0]]
    return x - torch.tensor(CAFFE_MEAN_BGR, dtype=x.dtype)


def maxpool_zero_padded(x, k=3, s=2, pad=1):
    """ZeroPadding2D(pad) + MaxPooling2D(k, s) (padding zeros take part in the max)."""
    return F.max_pool2d(F.pad(x, (pad, pad, pad, pad)), k, s)


def _relu(x, site, masks=None, branches=None):
    """ReLU at a named site (the HIP engine's buffer name for its output). masks: optional
    {site: [N,C,H,W] bool} replacing the ReLU by a multiplication with the given branch mask (the
    branches another implementation took, for comparing arithmetic where a pre-activation lies
    within rounding of 0); branches: optional dict receiving {site: x > 0} (this run's own)."""
    if branches is not None:
        if hasattr(branches, "record"):  # e.g. tests' FlipProbe: also sees the pre-activation
            branches.record(site, x.detach())
        else:
            branches[site] = (x > 0).detach()
    if masks is not None and site in masks:
        return x * masks[site].to(x.dtype)
    return torch.relu(x)


def relu_sites():
    """Every ReLU site of the forward, by the HIP engine's output-buffer name."""
    out = ["conv1_relu"]
    for name, f, blocks, stride1 in RESNET50_STACKS:
        for b in range(1, blocks + 1):
            pre = f"{name}_block{b}_"
            out += [pre + "1_relu", pre + "2_relu", pre + "out"]
    for name, *_ in FFLS:
        for part in ("block_left", "block_down"):
            for half in (0, 3):
                n = f"{name}/{part}"
                out += [f"{n}/act{half}", f"{n}/act{half + 1}", f"{n}/out{half}"]
    return out + ["aol/act0"]


def encoder(P, x, acts, masks=None, branches=None):
    """x: NCHW preprocessed input. Fills acts with every block output; returns the taps."""
    x = conv(x, P["conv1_conv/kernel"], P["conv1_conv/bias"], 2, (3, 3, 3, 3))
    x = _relu(_bn(P, "conv1_bn", x, RESNET_BN_EPS), "conv1_relu", masks, branches)
    acts["conv1_relu"] = x
    x = maxpool_zero_padded(x)
    acts["pool1_pool"] = x
    for name, f, blocks, stride1 in RESNET50_STACKS:
        for b in range(1, blocks + 1):
            pre = f"{name}_block{b}_"
            s = stride1 if b == 1 else 1
            if b == 1:
                sc = conv(x, P[pre + "0_conv/kernel"], P[pre + "0_conv/bias"], s)
                sc = _bn(P, pre + "0_bn", sc, RESNET_BN_EPS)
            else:
                sc = x
            y = conv(x, P[pre + "1_conv/kernel"], P[pre + "1_conv/bias"], s)
            y = _relu(_bn(P, pre + "1_bn", y, RESNET_BN_EPS), pre + "1_relu", masks, branches)
            y = conv_same(y, P[pre + "2_conv/kernel"], P[pre + "2_conv/bias"])
            y = _relu(_bn(P, pre + "2_bn", y, RESNET_BN_EPS), pre + "2_relu", masks, branches)
            y = conv(y, P[pre + "3_conv/kernel"], P[pre + "3_conv/bias"])
            y = _bn(P, pre + "3_bn", y, RESNET_BN_EPS)
            x = _relu(sc + y, pre + "out", masks, branches)
            acts[pre + "out"] = x
    return [acts[t] for t in TAPS]


def bottleneck(P, name, x, masks=None, branches=None):
    """BottleneckConvLayer.call (redweb.py:137-165)."""
    for half in (0, 3):
        res = x
        out = _relu(_bn(P, f"{name}/bn{half}", conv(x, P[f"{name}/conv{half}/kernel"]),
                        DEC_BN_EPS), f"{name}/act{half}", masks, branches)
        out = _relu(_bn(P, f"{name}/bn{half + 1}",
                        conv_same(out, P[f"{name}/conv{half + 1}/kernel"]), DEC_BN_EPS),
                    f"{name}/act{half + 1}", masks, branches)
        out = _bn(P, f"{name}/bn{half + 2}", conv(out, P[f"{name}/conv{half + 2}/kernel"]),
                  DEC_BN_EPS)
        x = _relu(out + res, f"{name}/out{half}", masks, branches)
    return x


def ffl(P, name, in_left, in_up, masks=None, branches=None):
    """FeatureFusionLayer.call (redweb.py:261-273)."""
    left = _bn(P, name + "/bn0", conv_same(in_left, P[name + "/conv0/kernel"]), DEC_BN_EPS)
    left = bottleneck(P, name + "/block_left", left, masks, branches)
    up = _bn(P, name + "/bn1", conv_same(in_up, P[name + "/conv1/kernel"]), DEC_BN_EPS)
    return up2(bottleneck(P, name + "/block_down", left + up, masks, branches))


def forward(P, x_nhwc, taps=None, preprocessed=False, relu_masks=None, relu_branches=None):
    """ff_redweb forward. P: fp64 tensors by name (param_specs). x_nhwc [N,H,W,3] in [0,1]
    (caffe preprocessing applied here unless preprocessed=True). relu_masks / relu_branches:
    as _relu, by relu_sites() name. Returns [N,H,W,1]."""
    acts = taps if taps is not None else {}
    if not preprocessed:
        x_nhwc = caffe_preprocess(x_nhwc)
    x = x_nhwc.permute(0, 3, 1, 2)
    g2, g3, g4, g5 = encoder(P, x, acts, relu_masks, relu_branches)
    b = up2(g5)
    for (name, _, _, _, _, _), left in zip(FFLS, (g4, g3, g2)):
        b = ffl(P, name, left, b, relu_masks, relu_branches)
        acts[name] = b
    x = conv_same(b, P["aol/conv0/kernel"], P["aol/conv0/bias"])
    x = _relu(_bn(P, "aol/bn0", x, DEC_BN_EPS), "aol/act0", relu_masks, relu_branches)
    x = conv_same(x, P["aol/conv1/kernel"], P["aol/conv1/bias"])
    x = up2(x)
    x = conv(x, P["aol/conv2/kernel"], P["aol/conv2/bias"])
    return x.permute(0, 2, 3, 1)


def trainable_names(P=None):
    return [n for n, _, kind in param_specs() if kind == "trainable"]


def train_step_grads(P, x_nhwc, dloss_dpred, preprocessed=False, relu_masks=None):
    names = set(trainable_names())
    Q = {k: (v.detach().clone().requires_grad_(True) if k in names else v.detach())
         for k, v in P.items()}
    out = forward(Q, x_nhwc, preprocessed=preprocessed, relu_masks=relu_masks)
    out.backward(dloss_dpred)
    return {k: Q[k].grad.detach() for k in names}, out.detach()


def conv_flops_per_image(H, W):
    """Algorithmic dense-conv FLOPs per image of one train step: fwd everywhere, dX through the
    encoder except the stem conv, dX + dW through the decoder (SURVEY §8d accounting)."""
    f = 0.0
    h, w = H // 2, W // 2
    f += h * w * 49 * 3 * 64  # stem fwd only
    h, w = h // 2, w // 2
    cin = 64
    for _, fl, blocks, stride1 in RESNET50_STACKS:
        for b in range(1, blocks + 1):
            s = stride1 if b == 1 else 1
            oh, ow = h // s, w // s
            if b == 1:
                f += 2 * oh * ow * cin * 4 * fl
            f += 2 * oh * ow * cin * fl + 2 * oh * ow * 9 * fl * fl + 2 * oh * ow * fl * 4 * fl
            cin, h, w = 4 * fl, oh, ow
    dec = 0.0
    sizes = {"ffl0": (H // 16, W // 16), "ffl1": (H // 8, W // 8), "ffl2": (H // 4, W // 4)}
    for name, inter, outp, _, cl, cu in FFLS:
        hh, ww = sizes[name]
        dec += hh * ww * 9 * (cl + cu) * inter
        for p in (inter, outp):
            q = p // 4
            dec += 2 * hh * ww * (p * q + 9 * q * q + q * p)
    hh, ww = H // 2, W // 2
    dec += hh * ww * 9 * 64 * 64 + hh * ww * 9 * 64 + H * W
    return 2.0 * (f + 3 * dec)
