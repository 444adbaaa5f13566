"""Building blocks shared by the HIP model engines (ff_effnet, ff_redweb): flat parameter
stores and Keras-named BatchNormalization / Conv2D wrappers around libpldepth_hip.so."""
import itertools

import numpy as np
import torch

from .. import kernels as K

_SEQ = itertools.count()  # creation order of stored tensors across an engine's stores

BN_EPS = 1e-3        # keras BatchNormalization defaults
BN_MOMENTUM = 0.99


class FlatStore:
    """Named views into one flat fp32 device buffer (16-byte aligned segments)."""

    def __init__(self):
        self.specs = []  # (name, shape, offset)
        self.order = {}  # name -> global creation index (graph order: keras_layout)
        self.size = 0
        self.buf = None
        self.views = {}

    def add(self, name, shape):
        n = int(np.prod(shape))
        self.specs.append((name, tuple(shape), self.size))
        self.order[name] = next(_SEQ)
        self.size += (n + 3) // 4 * 4
        return name

    def materialize(self, device):
        self.buf = torch.zeros(max(self.size, 4), dtype=torch.float32, device=device)
        for name, shape, off in self.specs:
            n = int(np.prod(shape))
            self.views[name] = self.buf[off:off + n].view(shape)
        return self

    def like(self):
        t = FlatStore()
        t.specs, t.size, t.order = self.specs, self.size, self.order
        return t

    def __getitem__(self, name):
        return self.views[name]

    def names(self):
        return [s[0] for s in self.specs]


class _BN:
    """One Keras BatchNormalization (training mode: batch statistics + moving-average update;
    inference: moving statistics)."""

    def __init__(self, eng, name, c, eps=BN_EPS, momentum=BN_MOMENTUM):
        self.name, self.c = name, c
        self.eps, self.momentum = eps, momentum
        self.g = eng.params.add(name + "/gamma", (c,))
        self.b = eng.params.add(name + "/beta", (c,))
        self.mm = eng.stats.add(name + "/moving_mean", (c,))
        self.mv = eng.stats.add(name + "/moving_variance", (c,))
        eng.bns.append(self)

    def bind(self, eng):
        dev = eng.device
        self.gamma, self.beta = eng.params[self.g], eng.params[self.b]
        self.dgamma, self.dbeta = eng.grads[self.g], eng.grads[self.b]
        self.mmean, self.mvar = eng.stats[self.mm], eng.stats[self.mv]
        self.mean = torch.empty(self.c, device=dev)
        self.invstd = torch.empty(self.c, device=dev)
        self.inf_scale = torch.empty(self.c, device=dev)
        self.inf_shift = torch.empty(self.c, device=dev)

    def stats_(self, x, rows, training):
        if training:
            K.bn_stats(x, rows, self.c, self.mean, self.invstd, self.mmean, self.mvar, self.eps,
                       self.momentum)
        else:
            K.bn_inference_coeffs(self.gamma, self.beta, self.mmean, self.mvar, self.inf_scale,
                                  self.inf_shift, self.eps)

    def conv_fwd_stats(self, args, w_nat, bias, y, rows, training):
        """conv forward into y, then this BN's statistics of y: in training they come from the
        conv kernel's epilogue where it supports it (pld_conv2d_fwd_bn_stats)."""
        if training:
            K.conv2d_fwd_bn_stats(args, w_nat, bias, y, self.mean, self.invstd, self.mmean,
                                  self.mvar, self.eps, self.momentum)
        else:
            K.conv2d_fwd(args, w_nat, bias, y)
            self.stats_(y, rows, False)

    def apply(self, x, rows, act, y, training, gate=None, hw=0):
        if training:
            K.bn_apply(x, rows, self.c, self.mean, self.invstd, self.gamma, self.beta, act, y,
                       gate=gate, hw=hw)
        else:
            assert gate is None
            K.channel_affine_act(x, rows, self.c, self.inf_scale, self.inf_shift, act, y)

    def bwd(self, x, dy, rows, act, dx, dx_acc=False, gate=None, addn=None, hw=0):
        K.bn_bwd(x, dy, rows, self.c, self.mean, self.invstd, self.gamma, self.beta, act, dx,
                 self.dgamma, self.dbeta, gate=gate, addn=addn, hw=hw, dx_accumulate=dx_acc)

    def add_apply(self, x, rows, res, act, y, training):
        """y = act(bn(x) + res)"""
        if training:
            K.bn_add_apply(x, rows, self.c, self.mean, self.invstd, self.gamma, self.beta, res,
                           act, y)
        else:
            if act == "none":
                K.channel_affine_act(x, rows, self.c, self.inf_scale, self.inf_shift, "none", y)
                K.residual_add(y, None, res, y)
            else:  # identity statistics turn bn_add_apply into act(z + res)
                K.channel_affine_act(x, rows, self.c, self.inf_scale, self.inf_shift, "none", y)
                z, o = _ident(self.c, x.device)
                K.bn_add_apply(y, rows, self.c, z, o, o, z, res, act, y)

    def add_bwd(self, x, dy, rows, res, act, dx, dres, dx_acc=False, dres_acc=False):
        K.bn_add_bwd(x, dy, rows, self.c, self.mean, self.invstd, self.gamma, self.beta, res, act,
                     dx, dres, self.dgamma, self.dbeta, dx_accumulate=dx_acc,
                     dres_accumulate=dres_acc)


_IDENT = {}


def _ident(c, device):
    """(zeros, ones) per channel count: a BN apply with these statistics is exact identity."""
    key = (c, str(device))
    if key not in _IDENT:
        _IDENT[key] = (torch.zeros(c, device=device), torch.ones(c, device=device))
    return _IDENT[key]


class _Conv:
    def __init__(self, eng, name, k, cin, cout, stride=1, bias=False, trainable=False,
                 need_dgrad=True):
        self.name, self.k, self.cin, self.cout, self.stride = name, k, cin, cout, stride
        self.has_bias, self.trainable, self.need_dgrad = bias, trainable, need_dgrad
        store = eng.params if trainable else eng.frozen
        self.wk = store.add(name + "/kernel", (k, k, cin, cout))
        self.bk = store.add(name + "/bias", (cout,)) if bias else None
        eng.convs.append(self)

    def bind(self, eng):
        store = eng.params if self.trainable else eng.frozen
        self.w = store[self.wk]
        self.b = store[self.bk] if self.bk else None
        if self.trainable:
            self.dw = eng.grads[self.wk]
            self.db = eng.grads[self.bk] if self.bk else None
        dev = eng.device
        self.w_nat = torch.empty(self.cout, self.k, self.k, self.cin, device=dev)
        self.w_dg = (torch.empty(self.cin, self.k, self.k, self.cout, device=dev)
                     if self.need_dgrad else None)
        # bf16x3 pre-split copies (fwd K = k*k*cin, dgrad K = k*k*cout must be multiples of 8)
        self.w_nat_x3 = torch.empty_like(self.w_nat) if self.cin % 8 == 0 else None
        self.w_dg_x3 = (torch.empty_like(self.w_dg)
                        if self.w_dg is not None and self.cout % 8 == 0 else None)

    def refresh(self):
        K.filter_refresh(self.w, self.w_nat, self.w_nat_x3, self.w_dg, self.w_dg_x3)


def refresh_trainable_convs(eng):
    """Every trainable conv's filter copies after the optimizer step, in one launch
    (kernels.FilterRefreshBatch over a device descriptor table of raw pointers). The table is
    built at the first call — an eager step always precedes a graph capture — and rebuilt when
    any conv's buffers were rebound since (the pointers it holds are compared with the convs'
    current tensors on every eager call), so it never writes through stale pointers; a capture
    that would need a rebuild fails instead."""
    entries = [(c.w, c.w_nat, c.w_nat_x3, c.w_dg, c.w_dg_x3) for c in eng.convs if c.trainable]
    key = [tuple(None if t is None else t.data_ptr() for t in e) for e in entries]
    batch = getattr(eng, "_refresh_batch", None)
    if batch is None or getattr(eng, "_refresh_key", None) != key:
        assert not K._CAPTURING[0], "the refresh table must be (re)built before graph capture"
        batch = eng._refresh_batch = K.FilterRefreshBatch(entries, eng.device)
        eng._refresh_key = key
    batch()
