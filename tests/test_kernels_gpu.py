"""GPU parity tests: every HIP kernel of libpldepth_hip.so against the CPU oracle.

Float kernels are checked against torch-CPU fp64 restatements (oracle/effnet.py helpers) with an
explicit tolerance; integer/index work (sampler) bit-exactly against oracle/sampler.py fed the
same draws.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import effnet as OE
from oracle import listmle as LM
from oracle import sampler as S
import ctypes as C

from pldepth_amd import _lib
from pldepth_amd import kernels as K

pytestmark = pytest.mark.gpu
RTOL = 1e-3  # BASELINE.json: 1e-3 relative on fp32 activations, loss and gradients
# conv tolerance per product arithmetic (pld_conv_args.math): exact fp32 MFMA lands ~1e-7 from
# fp64; bf16x3 (three bf16 products, |error| <= ~2^-16 per product) ~1e-5
CONV_TOL = {"fp32": 1e-5, "bf16x3": 1e-4}
MATHS = ["fp32", "bf16x3"]


def rel_err(got, ref):
    got = got.detach().double().cpu()
    ref = ref.detach().double().cpu()
    return float((got - ref).abs().max() / ref.abs().max().clamp(min=1e-30))


def dev(t, cuda):
    return t.to(device=cuda, dtype=torch.float32).contiguous()


# ------------------------------------------------------------------------------- ListMLE
@pytest.mark.parametrize("B,H,W,R,L", [(2, 8, 9, 5, 2), (3, 16, 16, 7, 5), (2, 12, 12, 6, 64),
                                       (1, 20, 20, 3, 130), (1, 30, 30, 2, 500)])
def test_listmle_matches_oracle(cuda, B, H, W, R, L):
    rng = np.random.default_rng(L)
    pred = rng.standard_normal((B, H, W, 1)).astype(np.float32)
    idx = rng.integers(0, H * W, (B, R, L))
    lab = (rng.permutation(B * R * L).reshape(B, R, L) / (B * R * L)).astype(np.float32)
    lab[0, 0, -1] = -1.0  # an invalid element
    y = np.stack([idx.astype(np.float32), lab], -1).astype(np.float32)
    loss_ref, dpred_ref = LM.hourglass_nll(y, pred, B, L)
    loss, dpred, nll = K.listmle_fwd_bwd(dev(torch.from_numpy(pred), cuda),
                                         dev(torch.from_numpy(y), cuda), B, R, L)
    torch.cuda.synchronize()
    assert abs(loss.item() - loss_ref) / abs(loss_ref) < 1e-5
    assert rel_err(dpred, torch.from_numpy(dpred_ref)) < 1e-5


def test_listmle_sorted_input_and_ties_deterministic(cuda):
    B, H, W, R, L = 2, 10, 10, 4, 5
    rng = np.random.default_rng(3)
    pred = rng.standard_normal((B, H, W, 1)).astype(np.float32)
    idx = rng.integers(0, H * W, (B, R, L))
    lab = np.sort(rng.integers(0, 4, (B, R, L)) / 4.0, axis=-1)[..., ::-1].astype(np.float32)
    y = np.ascontiguousarray(np.stack([idx.astype(np.float32), lab], -1))
    loss_ref, dpred_ref = LM.hourglass_nll(y, pred, B, L)
    loss, dpred, _ = K.listmle_fwd_bwd(dev(torch.from_numpy(pred), cuda),
                                       dev(torch.from_numpy(y), cuda), B, R, L)
    assert abs(loss.item() - loss_ref) / abs(loss_ref) < 1e-5
    assert rel_err(dpred, torch.from_numpy(dpred_ref)) < 1e-5


# ---------------------------------------------------------------------------------- Adam
def test_adam_amsgrad_matches_oracle(cuda):
    from oracle.adam import adam_amsgrad_step
    rng = np.random.default_rng(0)
    n = 1027
    p = rng.standard_normal(n).astype(np.float32)
    st = [np.zeros(n, np.float32) for _ in range(3)]
    tp = dev(torch.from_numpy(p), cuda)
    tm, tv, th = (torch.zeros(n, device=cuda) for _ in range(3))
    for step in range(1, 6):
        g = rng.standard_normal(n).astype(np.float32) * (0.1 if step % 2 else 3.0)
        p, *st = adam_amsgrad_step(p, g, *st, lr=0.01, step=step)
        K.adam_amsgrad(tp, dev(torch.from_numpy(g), cuda), tm, tv, th, lr=0.01, step=step)
    torch.cuda.synchronize()
    np.testing.assert_allclose(tp.cpu().numpy(), p, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(th.cpu().numpy(), st[2], rtol=1e-5, atol=1e-9)


# ---------------------------------------------------------------------------------- conv
CONV_CASES = [
    # n, h, w, c1, c2, k, s, cout, bias, prologue
    (2, 9, 11, 8, 12, 3, 1, 40, True, False),      # decoder-like: 3x3 same + concat
    (2, 7, 7, 16, 0, 1, 1, 96, False, False),      # 1x1 expand
    (1, 12, 10, 24, 0, 1, 1, 144, False, False),   # K=24 (not a multiple of 16)
    (2, 10, 12, 3, 0, 3, 2, 32, False, True),      # stem: Cin=3, s2, asymmetric pad, prologue
    (2, 16, 16, 32, 0, 3, 1, 1, True, False),      # final conv: Cout=1
    (1, 14, 14, 64, 64, 3, 1, 130, True, True),    # concat + prologue on source 1
    (2, 6, 6, 1280, 0, 3, 1, 672, True, False),    # c0-like channel counts
    (2, 37, 45, 16, 0, 3, 1, 1, True, False),      # Cout=1 direct kernels, ragged tiles
    (1, 40, 33, 32, 0, 3, 1, 1, False, False),
    (1, 10, 10, 12, 0, 3, 1, 1, True, False),      # Cout=1, C not a multiple of 8
    (2, 20, 18, 64, 0, 3, 1, 1, True, False),      # Cout=1, 64 channels (ReDWeb aol/conv1)
    (1, 17, 33, 36, 0, 3, 1, 1, False, False),     # Cout=1, ragged second channel chunk
    (16, 200, 200, 32, 0, 3, 1, 1, True, False),   # Cout=1, > 2048 tiles: persistent blocks
    (24, 150, 150, 36, 0, 3, 1, 1, False, False),  #   loop over several tiles (+ 2 chunks)
    (2, 12, 12, 48, 48, 3, 1, 144, True, False),   # N=144 (128x160 tile), dgrad N=96
    (1, 9, 9, 32, 64, 3, 1, 240, True, False),     # N=240; dgrad splits 32|64
    (1, 8, 8, 96, 0, 3, 1, 224, True, False),      # N=224 exact tile
    (3, 5, 7, 320, 0, 1, 1, 1280, False, False),   # top conv shape class
    (2, 37, 45, 1, 0, 1, 1, 1, True, False),       # 1 -> 1 channel 1x1 (ReDWeb aol/conv2):
    (4, 64, 64, 1, 0, 1, 1, 1, True, False),       #   scalar kernels, ragged and float4 tails
]


def _ref_conv(x1, x2, w, b, k, s, pt, pb, pl, pr, scale=None, shift=None):
    x = x1
    if scale is not None:
        x = torch.relu(x * scale + shift)
    if x2 is not None:
        x = torch.cat([x, x2], dim=-1)
    y = OE.conv(x.permute(0, 3, 1, 2), w, b, s, (pt, pb, pl, pr))
    return y.permute(0, 2, 3, 1)


@pytest.mark.parametrize("math", MATHS)
@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_fwd_dgrad_wgrad(cuda, case, math):
    tol = CONV_TOL[math]
    n, h, w, c1, c2, k, s, cout, has_bias, pro = case
    torch.manual_seed(hash(case) % 1000)
    x1 = torch.randn(n, h, w, c1, dtype=torch.float64)
    x2 = torch.randn(n, h, w, c2, dtype=torch.float64) if c2 else None
    wt = torch.randn(k, k, c1 + c2, cout, dtype=torch.float64) / np.sqrt(k * k * (c1 + c2))
    b = torch.randn(cout, dtype=torch.float64) if has_bias else None
    scale = torch.rand(c1, dtype=torch.float64) + 0.5 if pro else None
    shift = torch.randn(c1, dtype=torch.float64) * 0.3 if pro else None
    if s == 2:
        pt, pb = OE.correct_pad(h, k)
        pl, pr = OE.correct_pad(w, k)
    else:
        pt, pb, _ = OE.same_pad(h, k, 1)
        pl, pr, _ = OE.same_pad(w, k, 1)
    oh = (h + pt + pb - k) // s + 1
    ow = (w + pl + pr - k) // s + 1
    x1r = x1.clone().requires_grad_(True)
    x2r = x2.clone().requires_grad_(True) if x2 is not None else None
    wr = wt.clone().requires_grad_(True)
    y_ref = _ref_conv(x1r, x2r, wr, b, k, s, pt, pb, pl, pr, scale, shift)
    dy = torch.randn_like(y_ref)
    y_ref.backward(dy)

    gx1, gx2 = dev(x1, cuda), (dev(x2, cuda) if x2 is not None else None)
    gw = dev(wt, cuda)
    gsc = dev(scale, cuda) if pro else None
    gsh = dev(shift, cuda) if pro else None
    args = K.conv_args(gx1, gx2, k, k, s, pt, pl, oh, ow, cout, gsc, gsh,
                       "relu" if pro else "none", math=math)
    y = torch.empty(n, oh, ow, cout, device=cuda)
    K.conv2d_fwd(args, K.filter_to_native(gw), dev(b, cuda) if has_bias else None, y)
    torch.cuda.synchronize()
    assert rel_err(y, y_ref) < tol, rel_err(y, y_ref)
    # accumulate mode adds onto the destination
    K.conv2d_fwd(args, K.filter_to_native(gw), dev(b, cuda) if has_bias else None, y,
                 accumulate=True)
    assert rel_err(y, 2 * y_ref) < tol

    gdy = dev(dy, cuda)
    dw = torch.empty(k, k, c1 + c2, cout, device=cuda)
    K.conv2d_wgrad(args, gdy, dw)
    torch.cuda.synchronize()
    assert rel_err(dw, wr.grad) < tol, rel_err(dw, wr.grad)

    if s == 1 and not pro:
        dx1 = torch.empty_like(gx1)
        dx2 = torch.full_like(gx2, 1.0) if x2 is not None else None
        K.conv2d_dgrad(args, gdy, K.filter_to_dgrad(gw), dx1, dx2, acc2=True)
        torch.cuda.synchronize()
        assert rel_err(dx1, x1r.grad) < tol, rel_err(dx1, x1r.grad)
        if x2 is not None:
            assert rel_err(dx2 - 1.0, x2r.grad) < tol


@pytest.mark.parametrize("math", MATHS)
@pytest.mark.parametrize("n,h,w,c,cout", [(2, 14, 12, 64, 128), (1, 9, 11, 32, 48),
                                          (2, 7, 7, 6, 8)])
def test_conv_dgrad_strided_1x1(cuda, math, n, h, w, c, cout):
    """dgrad of a stride-2 1x1 conv (ResNet projection shortcuts / first 1x1 of a stage): the
    GEMM on the output grid, then the scatter into the input grid (zeros off the stride grid),
    overwrite and accumulate; odd input sizes; C % 4 != 0 takes the generic scatter."""
    torch.manual_seed(n * h + c)
    x = torch.randn(n, h, w, c, dtype=torch.float64, requires_grad=True)
    wt = torch.randn(1, 1, c, cout, dtype=torch.float64) / np.sqrt(c)
    oh, ow = (h - 1) // 2 + 1, (w - 1) // 2 + 1
    y = OE.conv(x.permute(0, 3, 1, 2), wt, None, 2, (0, 0, 0, 0)).permute(0, 2, 3, 1)
    assert y.shape[1:3] == (oh, ow)
    dy = torch.randn_like(y)
    y.backward(dy)
    gx = dev(x.detach(), cuda)
    args = K.conv_args(gx, None, 1, 1, 2, 0, 0, oh, ow, cout, math=math)
    dx = torch.full_like(gx, 0.25)
    K.conv2d_dgrad(args, dev(dy, cuda), K.filter_to_dgrad(dev(wt, cuda)), dx, acc1=True)
    torch.cuda.synchronize()
    assert rel_err(dx - 0.25, x.grad) < CONV_TOL[math]
    K.conv2d_dgrad(args, dev(dy, cuda), K.filter_to_dgrad(dev(wt, cuda)), dx)
    torch.cuda.synchronize()
    assert rel_err(dx, x.grad) < CONV_TOL[math]


@pytest.mark.parametrize("math", MATHS)
@pytest.mark.parametrize("case", [(2, 14, 14, 96, 32, 3, 1, 64, True),
                                  (1, 9, 11, 64, 0, 1, 1, 320, False),
                                  (2, 10, 9, 48, 24, 3, 1, 136, True),
                                  (2, 12, 10, 32, 16, 3, 1, 144, False),
                                  # the bf16x3 patch kernel: fwd of a 32-channel input (ragged
                                  # 8 x 32 tiles, N = 72: two N tiles at BN 64), dgrad with
                                  # dY of 32 channels routed to a 48 | 24 concat
                                  (2, 13, 40, 32, 0, 3, 1, 72, True),
                                  (2, 11, 35, 48, 24, 3, 1, 32, True),
                                  # the 64-cout patch WGRAD (dec1-like: concat of 32-channel
                                  # chunks with a ragged 16-channel one, N = 240, 28 x 28)
                                  (2, 28, 28, 64, 48, 3, 1, 240, False),
                                  # its 4-row tiles with ragged rows, columns and a ragged
                                  # second cout tile (N = 112: 64 + 48)
                                  (1, 15, 37, 32, 16, 3, 1, 112, False)])
def test_conv_every_schedule(cuda, case, math):
    """Each tile x split-K schedule computes the same conv (fwd with bias routing, dgrad into
    two concat destinations with accumulate)."""
    n, h, w, c1, c2, k, s, cout, has_bias = case
    torch.manual_seed(7)
    x1 = torch.randn(n, h, w, c1, dtype=torch.float64)
    x2 = torch.randn(n, h, w, c2, dtype=torch.float64) if c2 else None
    wt = torch.randn(k, k, c1 + c2, cout, dtype=torch.float64) / np.sqrt(k * k * (c1 + c2))
    b = torch.randn(cout, dtype=torch.float64) if has_bias else None
    pt, pb, _ = OE.same_pad(h, k, 1)
    pl, pr, _ = OE.same_pad(w, k, 1)
    x1r = x1.clone().requires_grad_(True)
    x2r = x2.clone().requires_grad_(True) if x2 is not None else None
    wr = wt.clone().requires_grad_(True)
    y_ref = _ref_conv(x1r, x2r, wr, b, k, 1, pt, pb, pl, pr)
    dy = torch.randn_like(y_ref)
    y_ref.backward(dy)
    gx1, gx2, gw = dev(x1, cuda), (dev(x2, cuda) if c2 else None), dev(wt, cuda)
    wn, wd = K.filter_to_native(gw), K.filter_to_dgrad(gw)
    gb, gdy = (dev(b, cuda) if has_bias else None), dev(dy, cuda)
    tol = CONV_TOL[math]
    n_sched = _lib.lib().pld_conv_num_schedules(K.MATH[math])
    assert n_sched >= 2
    for t in range(n_sched):
        args = K.conv_args(gx1, gx2, k, k, 1, pt, pl, h, w, cout, math=math)
        args.tile = t
        y = torch.full((n, h, w, cout), 0.5, device=cuda)
        K.conv2d_fwd(args, wn, gb, y, accumulate=True)
        dx1 = torch.empty_like(gx1)
        dx2 = torch.full_like(gx2, 1.0) if c2 else None
        K.conv2d_dgrad(args, gdy, wd, dx1, dx2, acc2=True)
        dw = torch.empty(k, k, c1 + c2, cout, device=cuda)
        K.conv2d_wgrad(args, gdy, dw)
        torch.cuda.synchronize()
        assert rel_err(y - 0.5, y_ref) < tol, (t, rel_err(y - 0.5, y_ref))
        assert rel_err(dx1, x1r.grad) < tol, t
        if c2:
            assert rel_err(dx2 - 1.0, x2r.grad) < tol, t
        assert rel_err(dw, wr.grad) < tol, t
    # a split-K schedule without a workspace fails loudly
    args = K.conv_args(gx1, gx2, k, k, 1, pt, pl, h, w, cout, math=math)
    args.tile = n_sched - 1
    need = _lib.lib().pld_conv2d_fwd_workspace_size(C.byref(args))
    if need:
        with pytest.raises(_lib.PLDError):
            _lib.lib().pld_conv2d_fwd(C.byref(args), wn.data_ptr(), None,
                                      torch.empty(n, h, w, cout, device=cuda).data_ptr(), 0, None)


@pytest.mark.parametrize("case", [
    # dec0-like: 14-wide map, 12 chunks (split-K into 3 x 4 chunks), bias, N tail
    (2, 14, 14, 320, 64, 200, True),
    # dec1-like: 28 x 28 concat of two ragged (16-channel tail) sources, N = 240
    (2, 28, 28, 80, 48, 240, False),
    # dec2-like: the widest map the kernel takes (56), patch rows = BM + 114
    (1, 56, 56, 96, 0, 144, True),
    # a band straddling images on a map narrower than a tile row, odd width and height
    (3, 9, 13, 40, 24, 72, True),
    # tile streams with >= 2 tiles per workgroup: the interleaved tile order (sk_perm 2 and 4,
    # a non-permuted tail tile)
    (2, 28, 28, 48, 0, 64, False),
    (4, 56, 56, 32, 0, 40, True)])
def test_conv_halo_schedules(cuda, case):
    """The row-band halo kernel (every x3halo / x3halosplit schedule): fwd with bias and
    accumulate, dgrad into a concat's two destinations (one accumulating), against fp64; the
    kernel names the call reports (pld_conv_kernel_name) are the halo kernel's."""
    n, h, w, c1, c2, cout, has_bias = case
    torch.manual_seed(11)
    x1 = torch.randn(n, h, w, c1, dtype=torch.float64)
    x2 = torch.randn(n, h, w, c2, dtype=torch.float64) if c2 else None
    wt = torch.randn(3, 3, c1 + c2, cout, dtype=torch.float64) / np.sqrt(9 * (c1 + c2))
    b = torch.randn(cout, dtype=torch.float64) if has_bias else None
    x1r = x1.clone().requires_grad_(True)
    x2r = x2.clone().requires_grad_(True) if x2 is not None else None
    y_ref = _ref_conv(x1r, x2r, wt, b, 3, 1, 1, 1, 1, 1)
    dy = torch.randn_like(y_ref)
    y_ref.backward(dy)
    gx1, gx2 = dev(x1, cuda), (dev(x2, cuda) if c2 else None)
    gw = dev(wt, cuda)
    wn, wd = K.filter_to_native(gw), K.filter_to_dgrad(gw)
    K.filter_split(wn, torch.empty_like(wn))
    gb, gdy = (dev(b, cuda) if has_bias else None), dev(dy, cuda)
    m = K.MATH["bf16x3"]
    halo = [t for t in range(_lib.lib().pld_conv_num_schedules(m))
            if _lib.lib().pld_conv_schedule_class(m, t) == 6]
    assert len(halo) >= 2 and all(K.schedule_desc(m, t).startswith("x3halo") for t in halo)
    for t in halo:
        args = K.conv_args(gx1, gx2, 3, 3, 1, 1, 1, h, w, cout, math="bf16x3")
        args.tile = t
        # the "x3halo28" schedules take maps up to 28 wide (wider ones run the default tile)
        want = (b"conv_x3_kernel" if "halo28" in K.schedule_desc(m, t) and w > 28
                else b"conv_x3_halo_kernel")
        for mode in (0, 1):
            assert _lib.lib().pld_conv_kernel_name(C.byref(args), mode) == want
        y = torch.full((n, h, w, cout), 0.5, device=cuda)
        K.conv2d_fwd(args, wn, gb, y, accumulate=True)
        dx1 = torch.empty_like(gx1)
        dx2 = torch.full_like(gx2, 1.0) if c2 else None
        K.conv2d_dgrad(args, gdy, wd, dx1, dx2, acc2=True)
        torch.cuda.synchronize()
        name = K.schedule_desc(m, t)
        assert rel_err(y - 0.5, y_ref) < CONV_TOL["bf16x3"], (name, rel_err(y - 0.5, y_ref))
        assert rel_err(dx1, x1r.grad) < CONV_TOL["bf16x3"], name
        if c2:
            assert rel_err(dx2 - 1.0, x2r.grad) < CONV_TOL["bf16x3"], name


@pytest.mark.parametrize("case", [
    # 1x1 on a 2 x 128 x 128 map: enough tiles to give workgroups several whole tiles (aligned
    # ranges: the pipeline runs on across tile boundaries); its wgrad (K = 32768 pixels) cuts
    # each tile over dozens of workgroups (fixup sums)
    (2, 128, 128, 192, 0, 1, 160, True),
    # dec_conv0-like 3x3 concat at 14 x 14 with long K (K = 11520): few tiles, stream-K cuts
    (2, 14, 14, 640, 640, 3, 336, True),
    # ragged everything: M, N and K tails, concat with a 16-channel chunk
    (3, 11, 13, 48, 16, 3, 72, False),
    # long K (32 steps) with more tiles than resident slots on some tiles (64x192 / 256x32: 576
    # tiles on 512 slots, two whole tiles per workgroup) and fewer on others (stream-K cuts)
    (2, 96, 96, 1024, 0, 1, 256, True)])
def test_conv_tile_stream(cuda, case):
    """The bf16x3 tile-stream schedules (conv_x3_kernel STREAM + x3_stream_fixup_kernel): fwd
    (+bias, accumulate), dgrad into two concat destinations (accumulate on one), wgrad, and the
    fused BN statistics of the forward (in the main kernel's epilogue for whole tiles, in the
    fixup for cut ones) against fp64 / the unfused statistics pass."""
    n, h, w, c1, c2, k, cout, has_bias = case
    torch.manual_seed(11)
    x1 = torch.randn(n, h, w, c1, dtype=torch.float64)
    x2 = torch.randn(n, h, w, c2, dtype=torch.float64) if c2 else None
    wt = torch.randn(k, k, c1 + c2, cout, dtype=torch.float64) / np.sqrt(k * k * (c1 + c2))
    b = torch.randn(cout, dtype=torch.float64) if has_bias else None
    pt, pb, _ = OE.same_pad(h, k, 1)
    pl, pr, _ = OE.same_pad(w, k, 1)
    x1r = x1.clone().requires_grad_(True)
    x2r = x2.clone().requires_grad_(True) if x2 is not None else None
    wr = wt.clone().requires_grad_(True)
    y_ref = _ref_conv(x1r, x2r, wr, b, k, 1, pt, pb, pl, pr)
    dy = torch.randn_like(y_ref)
    y_ref.backward(dy)
    gx1, gx2, gw = dev(x1, cuda), (dev(x2, cuda) if c2 else None), dev(wt, cuda)
    wn, wd = K.filter_to_native(gw), K.filter_to_dgrad(gw)
    gb, gdy = (dev(b, cuda) if has_bias else None), dev(dy, cuda)
    lib = _lib.lib()
    m = K.MATH["bf16x3"]
    streams = [t for t in range(lib.pld_conv_num_schedules(m))
               if lib.pld_conv_schedule_class(m, t) == 5]
    assert streams and all(K.schedule_desc(m, t).startswith("x3stream/") for t in streams)
    rows = n * h * w
    for t in streams:
        args = K.conv_args(gx1, gx2, k, k, 1, pt, pl, h, w, cout, math="bf16x3")
        args.tile = t
        assert K.conv_kernel_name(args, "fwd") == "conv_x3_kernel"
        y = torch.full((n, h, w, cout), 0.5, device=cuda)
        K.conv2d_fwd(args, wn, gb, y, accumulate=True)
        dx1 = torch.empty_like(gx1)
        dx2 = torch.full_like(gx2, 1.0) if c2 else None
        K.conv2d_dgrad(args, gdy, wd, dx1, dx2, acc2=True)
        dw = torch.empty(k, k, c1 + c2, cout, device=cuda)
        K.conv2d_wgrad(args, gdy, dw)
        y2 = torch.empty(n, h, w, cout, device=cuda)
        mean, inv = torch.empty(cout, device=cuda), torch.empty(cout, device=cuda)
        K.conv2d_fwd_bn_stats(args, wn, gb, y2, mean, inv)
        torch.cuda.synchronize()
        desc = K.schedule_desc(m, t)
        assert rel_err(y - 0.5, y_ref) < 1e-4, (desc, rel_err(y - 0.5, y_ref))
        assert torch.equal(y2, y - 0.5) or rel_err(y2, y_ref) < 1e-4, desc
        assert rel_err(dx1, x1r.grad) < 1e-4, desc
        if c2:
            assert rel_err(dx2 - 1.0, x2r.grad) < 1e-4, desc
        assert rel_err(dw, wr.grad) < 1e-4, (desc, rel_err(dw, wr.grad))
        m_ref, i_ref = torch.empty(cout, device=cuda), torch.empty(cout, device=cuda)
        K.bn_stats(y2, rows, cout, m_ref, i_ref)
        torch.cuda.synchronize()
        assert rel_err(mean, m_ref) < 1e-6 and rel_err(inv, i_ref) < 1e-6, desc


@pytest.mark.parametrize("math", MATHS)
@pytest.mark.parametrize("case", [(2, 14, 12, 64, 3, 96, "relu"), (1, 9, 11, 256, 1, 64, "relu"),
                                  (2, 10, 9, 32, 3, 48, "swish"), (2, 7, 9, 128, 3, 130, "relu"),
                                  (3, 5, 7, 512, 1, 200, "none")])
def test_conv_prologue_every_schedule(cuda, case, math):
    """The fused input prologue y = conv(act(x*scale + shift)) (a BatchNorm apply + activation
    of the producing layer, never materialised) on every schedule of a one-source conv: padding
    taps stay zero after the activation (they are not act(shift)); tap-inner (3x3, C >= 64),
    linear (3x3 on 32 channels) and 1x1 K orders, ragged M and N tiles."""
    n, h, w, c, k, cout, act = case
    torch.manual_seed(c + cout)
    x = torch.randn(n, h, w, c, dtype=torch.float64)
    wt = torch.randn(k, k, c, cout, dtype=torch.float64) / np.sqrt(k * k * c)
    scale = torch.rand(c, dtype=torch.float64) + 0.5
    shift = torch.randn(c, dtype=torch.float64) * 0.5
    z = x * scale + shift
    a = {"relu": torch.relu(z), "swish": z * torch.sigmoid(z), "none": z}[act]
    pt, pb, _ = OE.same_pad(h, k, 1)
    pl, pr, _ = OE.same_pad(w, k, 1)
    y_ref = OE.conv(a.permute(0, 3, 1, 2), wt, None, 1, (pt, pb, pl, pr)).permute(0, 2, 3, 1)
    gx, gw = dev(x, cuda), dev(wt, cuda)
    wn = K.filter_to_native(gw)
    gsc, gsh = dev(scale, cuda), dev(shift, cuda)
    tol = CONV_TOL[math]
    n_sched = _lib.lib().pld_conv_num_schedules(K.MATH[math])
    for t in list(range(n_sched)) + [-1]:
        args = K.conv_args(gx, None, k, k, 1, pt, pl, h, w, cout, gsc, gsh, act, math=math)
        args.tile = t
        ws = torch.empty(max(_lib.lib().pld_conv2d_fwd_workspace_size(C.byref(args)), 4),
                         dtype=torch.uint8, device=cuda)
        args.ws, args.ws_bytes = ws.data_ptr(), ws.numel()
        y = torch.empty(n, h, w, cout, device=cuda)
        _lib.lib().pld_conv2d_fwd(C.byref(args), wn.data_ptr(), None, y.data_ptr(), 0, None)
        torch.cuda.synchronize()
        assert rel_err(y, y_ref) < tol, (t, rel_err(y, y_ref))


@pytest.mark.parametrize("math", MATHS)
@pytest.mark.parametrize("k,cout,cpad,norm", [(3, 32, 8, True), (7, 64, 8, False),
                                             (3, 32, 4, True), (7, 64, 4, False)])
def test_padded_stem(cuda, math, k, cout, cpad, norm):
    """The stems' widened input: pld_channel_pad_affine (normalisation + zero channels) then the
    stride-2 conv with a zero-padded filter equals the 3-channel conv of the normalised input
    (EfficientNetB0 3x3 TF-SAME / ResNet-50 7x7 pad 3; padding taps zero either way)."""
    torch.manual_seed(k * cpad)
    n, h, w = 2, 30, 26
    x = torch.rand(n, h, w, 3, dtype=torch.float64) * 255
    wt = torch.randn(k, k, 3, cout, dtype=torch.float64) / np.sqrt(k * k * 3)
    sc = torch.tensor([0.017, 0.018, 0.0175], dtype=torch.float64) if norm else None
    sh = torch.tensor([-2.1, -2.0, -1.8], dtype=torch.float64) if norm else None
    xn = x * sc + sh if norm else x
    if k == 3:
        pt, pb = OE.correct_pad(h, k)
        pl, pr = OE.correct_pad(w, k)
    else:
        pt = pb = pl = pr = 3
    oh, ow = (h + pt + pb - k) // 2 + 1, (w + pl + pr - k) // 2 + 1
    y_ref = OE.conv(xn.permute(0, 3, 1, 2), wt, None, 2, (pt, pb, pl, pr)).permute(0, 2, 3, 1)
    gx = dev(x, cuda)
    xp = torch.full((n, h, w, cpad), 7.0, device=cuda)  # stale contents must be overwritten
    K.channel_pad_affine(gx, cpad, xp, dev(sc, cuda) if norm else None,
                         dev(sh, cuda) if norm else None)
    torch.cuda.synchronize()
    assert torch.all(xp[..., 3:] == 0)
    assert rel_err(xp[..., :3], xn) < 1e-6
    wp = torch.zeros(k, k, cpad, cout, dtype=torch.float64)
    wp[:, :, :3] = wt
    args = K.conv_args(xp, None, k, k, 2, pt, pl, oh, ow, cout, math=math)
    wn = K.filter_to_native(dev(wp, cuda))
    if math == "bf16x3" and cpad % 8 == 0:
        K.filter_split(wn)
    y = torch.empty(n, oh, ow, cout, device=cuda)
    K.conv2d_fwd(args, wn, None, y)
    torch.cuda.synchronize()
    assert rel_err(y, y_ref) < CONV_TOL[math], rel_err(y, y_ref)


def test_bn_train_coeffs(cuda):
    """scale = gamma*invstd, shift = beta - mean*scale: act(x*scale + shift) == bn_apply."""
    torch.manual_seed(3)
    rows, c = 777, 40
    x = torch.randn(rows, c, device=cuda) * 3 + 1
    mean, invstd = torch.empty(c, device=cuda), torch.empty(c, device=cuda)
    K.bn_stats(x, rows, c, mean, invstd)
    gamma, beta = torch.rand(c, device=cuda) + 0.5, torch.randn(c, device=cuda)
    sc, sh = torch.empty(c, device=cuda), torch.empty(c, device=cuda)
    K.bn_train_coeffs(mean, invstd, gamma, beta, sc, sh)
    y = torch.empty_like(x)
    K.bn_apply(x, rows, c, mean, invstd, gamma, beta, "relu", y)
    torch.cuda.synchronize()
    assert rel_err(torch.relu(x * sc + sh), y) < 1e-6


def test_channel_sum(cuda):
    x = torch.randn(1000, 37, dtype=torch.float64)
    out = torch.empty(37, device=cuda)
    K.channel_sum(dev(x, cuda), 1000, 37, out)
    assert rel_err(out, x.sum(0)) < 1e-6
    x = torch.randn(5003, 64, dtype=torch.float64)
    out = torch.ones(64, device=cuda)
    K.channel_sum(dev(x, cuda), 5003, 64, out, accumulate=True)
    assert rel_err(out - 1, x.sum(0)) < 1e-5


# ------------------------------------------------------------------------------------ BN
@pytest.mark.parametrize("rows,c,act", [(4096, 32, "relu"), (999, 144, "swish"),
                                        (300, 1280, "swish"), (50, 6, "none"),
                                        # two channel columns of 84 groups (red_plan)
                                        (3001, 672, "swish"),
                                        # grid-stride apply loops (> 8192 x 256 vectors): the
                                        # grid is a multiple of C / VW groups per thread
                                        (100003, 96, "swish"), (2100007, 3, "relu")])
def test_bn_forward_backward(cuda, rows, c, act):
    torch.manual_seed(rows + c)
    x = torch.randn(rows, c, dtype=torch.float64) * 3 + 1.5
    gamma = torch.rand(c, dtype=torch.float64) + 0.5
    beta = torch.randn(c, dtype=torch.float64)
    xr, gr, br = (t.clone().requires_grad_(True) for t in (x, gamma, beta))
    mean = xr.mean(0)
    var = ((xr - mean) ** 2).mean(0)
    z = (xr - mean) / torch.sqrt(var + 1e-3) * gr + br
    y_ref = {"relu": torch.relu, "swish": lambda t: t * torch.sigmoid(t),
             "none": lambda t: t}[act](z)
    dy = torch.randn_like(y_ref)
    y_ref.backward(dy)

    gx = dev(x, cuda)
    gm, gi = torch.empty(c, device=cuda), torch.empty(c, device=cuda)
    mm, mv = torch.zeros(c, device=cuda), torch.ones(c, device=cuda)
    K.bn_stats(gx, rows, c, gm, gi, mm, mv)
    y = torch.empty_like(gx)
    K.bn_apply(gx, rows, c, gm, gi, dev(gamma, cuda), dev(beta, cuda), act, y)
    torch.cuda.synchronize()
    assert rel_err(y, y_ref) < 1e-5
    uvar = x.var(0, unbiased=True)
    assert rel_err(mm, 0.01 * x.mean(0)) < 1e-5
    assert rel_err(mv, 0.99 + 0.01 * uvar) < 1e-5
    dx = torch.empty_like(gx)
    dg, db = torch.empty(c, device=cuda), torch.empty(c, device=cuda)
    K.bn_bwd(gx, dev(dy, cuda), rows, c, gm, gi, dev(gamma, cuda), dev(beta, cuda), act, dx, dg,
             db)
    torch.cuda.synchronize()
    assert rel_err(dx, xr.grad) < 1e-4, rel_err(dx, xr.grad)
    assert rel_err(dg, gr.grad) < 1e-5
    assert rel_err(db, br.grad) < 1e-5


@pytest.mark.parametrize("rows,c", [(401408, 24), (6272, 1152), (777, 40)])
def test_bn_reductions_repeat_bitwise(cuda, rows, c):
    """BN statistics, BN backward and the channel sum (fp64 partials, fixed-order finalize):
    repeated eager launches and replays of a captured graph give bit-identical statistics,
    coefficients and gradients, one and two channel columns, tens to thousands of partials."""
    g = torch.Generator(device=cuda).manual_seed(rows + c)
    x = torch.randn(rows, c, device=cuda, generator=g) * 2 + 0.5
    dy = torch.randn(rows, c, device=cuda, generator=g)
    gamma = torch.rand(c, device=cuda, generator=g) + 0.5
    beta = torch.randn(c, device=cuda, generator=g)
    outs = [torch.empty(c, device=cuda) for _ in range(4)] + [torch.empty_like(x)] + \
        [torch.empty(c, device=cuda)]
    gm, gi, dg, db, dx, cs = outs

    def run():
        K.bn_stats(x, rows, c, gm, gi)
        K.bn_bwd(x, dy, rows, c, gm, gi, gamma, beta, "swish", dx, dg, db)
        K.channel_sum(dy, rows, c, cs)

    run()
    torch.cuda.synchronize()
    ref = [t.clone() for t in outs]
    x64, dy64 = x.double(), dy.double()
    assert rel_err(gm, x64.mean(0)) < 1e-6
    assert rel_err(cs, dy64.sum(0)) < 1e-5
    for _ in range(2):
        for t in outs:
            t.fill_(float("nan"))
        run()
        torch.cuda.synchronize()
        assert all(torch.equal(a, b) for a, b in zip(outs, ref))
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        gr = K.Graph().capture(run)
        for _ in range(3):
            for t in outs:
                t.fill_(float("nan"))
            gr.launch()
            st.synchronize()
            assert all(torch.equal(a, b) for a, b in zip(outs, ref))
    del gr


def test_bn_with_se_gate_and_addn(cuda):
    n, hw, c = 3, 50, 16
    rows = n * hw
    torch.manual_seed(5)
    x = torch.randn(rows, c, dtype=torch.float64)
    gamma, beta = torch.rand(c, dtype=torch.float64) + .5, torch.randn(c, dtype=torch.float64)
    gate = torch.rand(n, c, dtype=torch.float64)
    addn = torch.randn(n, c, dtype=torch.float64) * 0.1
    xr, gr, br = (t.clone().requires_grad_(True) for t in (x, gamma, beta))
    mean = xr.mean(0)
    var = ((xr - mean) ** 2).mean(0)
    a = (xr - mean) / torch.sqrt(var + 1e-3) * gr + br
    a = a * torch.sigmoid(a)
    y_ref = a.view(n, hw, c) * gate.view(n, 1, c)
    dy = torch.randn(n, hw, c, dtype=torch.float64)
    # da = dy*gate + addn (the SE backward contract)
    (a.view(n, hw, c) * (dy * gate.view(n, 1, c) + addn.view(n, 1, c))).sum().backward()
    gx = dev(x, cuda)
    gm, gi = torch.empty(c, device=cuda), torch.empty(c, device=cuda)
    K.bn_stats(gx, rows, c, gm, gi)
    y = torch.empty_like(gx)
    K.bn_apply(gx, rows, c, gm, gi, dev(gamma, cuda), dev(beta, cuda), "swish", y,
               gate=dev(gate, cuda), hw=hw)
    assert rel_err(y.view(n, hw, c), y_ref) < 1e-5
    dx = torch.empty_like(gx)
    dg, db = torch.empty(c, device=cuda), torch.empty(c, device=cuda)
    K.bn_bwd(gx, dev(dy.reshape(rows, c), cuda), rows, c, gm, gi, dev(gamma, cuda),
             dev(beta, cuda), "swish", dx, dg, db, gate=dev(gate, cuda), addn=dev(addn, cuda),
             hw=hw)
    torch.cuda.synchronize()
    assert rel_err(dx, xr.grad) < 1e-4
    assert rel_err(dg, gr.grad) < 1e-5


# ---------------------------------------------------------------------------- resampling
@pytest.mark.parametrize("n,h,w,c", [(2, 5, 7, 8), (1, 1, 3, 4), (2, 14, 14, 672), (1, 4, 4, 3)])
def test_upsample2x(cuda, n, h, w, c):
    x = torch.randn(n, h, w, c, dtype=torch.float64, requires_grad=True)
    y_ref = OE.up2(x.permute(0, 3, 1, 2)).permute(0, 2, 3, 1)
    dy = torch.randn_like(y_ref)
    y_ref.backward(dy)
    y = torch.empty(n, 2 * h, 2 * w, c, device=cuda)
    K.upsample2x_fwd(dev(x.detach(), cuda), y)
    dx = torch.empty(n, h, w, c, device=cuda)
    K.upsample2x_bwd(dev(dy, cuda), dx)
    torch.cuda.synchronize()
    assert rel_err(y, y_ref) < 1e-6
    assert rel_err(dx, x.grad) < 1e-6


@pytest.mark.parametrize("n,h,w,c", [(2, 5, 7, 8), (1, 4, 4, 3), (2, 14, 14, 144)])
def test_upsample2x_bn_prologue(cuda, n, h, w, c):
    """decoder training forward: BN + ReLU of the conv output applied inside the upsample"""
    x = torch.randn(n, h, w, c, dtype=torch.float64)
    gamma, beta = torch.rand(c, dtype=torch.float64) + 0.5, torch.randn(c, dtype=torch.float64)
    rows = n * h * w
    gx = dev(x, cuda)
    gm, gi = torch.empty(c, device=cuda), torch.empty(c, device=cuda)
    K.bn_stats(gx, rows, c, gm, gi)
    mu, var = x.mean((0, 1, 2)), x.var((0, 1, 2), unbiased=False)
    a = torch.relu((x - mu) / torch.sqrt(var + 1e-3) * gamma + beta)
    y_ref = OE.up2(a.permute(0, 3, 1, 2)).permute(0, 2, 3, 1)
    y = torch.empty(n, 2 * h, 2 * w, c, device=cuda)
    K.upsample2x_fwd(gx, y, bn=(gm, gi, dev(gamma, cuda), dev(beta, cuda)), act="relu")
    # the fused form must equal the two-pass form (bn_apply then upsample) to the last bit
    act = torch.empty_like(gx)
    K.bn_apply(gx, rows, c, gm, gi, dev(gamma, cuda), dev(beta, cuda), "relu", act)
    y2 = torch.empty_like(y)
    K.upsample2x_fwd(act, y2)
    torch.cuda.synchronize()
    assert rel_err(y, y_ref) < 1e-5
    assert rel_err(y, y2) < 1e-6


def test_residual_and_per_sample_scale(cuda):
    a = torch.randn(3, 4, 5, 8)
    b = torch.randn(3, 4, 5, 8)
    sc = torch.tensor([0.0, 1.25, 1.25])
    y = torch.empty(3, 4, 5, 8, device=cuda)
    K.residual_add(a.to(cuda), sc.to(cuda), b.to(cuda), y)
    # bit for bit the two-step fp32 form (Keras: Dropout's product rounded, then Add's sum)
    torch.testing.assert_close(y.cpu(), a * sc.view(3, 1, 1, 1) + b, rtol=0, atol=0)
    K.scale_per_sample(a.to(cuda), sc.to(cuda), y, accumulate=True)
    torch.testing.assert_close(y.cpu(), 2 * a * sc.view(3, 1, 1, 1) + b)


@pytest.mark.parametrize("shape", [(3, 4, 5, 8), (2, 3, 5, 3), (4, 7, 7, 24)])
def test_residual_inplace_vector_and_scalar_paths(cuda, shape):
    """float4 path (per-image size % 4 == 0) and the scalar path, in place (y is a) as the
    engine calls it, with and without the per-sample drop-connect scale."""
    a = torch.randn(*shape)
    b = torch.randn(*shape)
    sc = torch.rand(shape[0]) + 0.5
    ga = a.to(cuda)
    K.residual_add(ga, sc.to(cuda), b.to(cuda), ga)
    torch.testing.assert_close(ga.cpu(), a * sc.view(-1, 1, 1, 1) + b, rtol=0, atol=0)
    gb = a.to(cuda)
    K.residual_add(gb, None, b.to(cuda), gb)
    torch.testing.assert_close(gb.cpu(), a + b)


# ------------------------------------------------------------------------- depthwise / SE
@pytest.mark.parametrize("n,h,w,c,k,s", [(2, 12, 12, 16, 3, 1), (2, 12, 10, 24, 3, 2),
                                         (1, 14, 14, 40, 5, 2), (2, 7, 7, 8, 5, 1),
                                         (1, 13, 11, 4, 3, 2), (1, 9, 13, 12, 5, 1),
                                         (2, 15, 17, 8, 5, 2), (1, 5, 6, 4, 3, 1),
                                         # the LDS-tiled kernel (c % 16 == 0): 4- and 8-quad
                                         # channel groups, ragged tiles, both strides
                                         (2, 37, 21, 48, 5, 1), (1, 35, 19, 64, 3, 2),
                                         (2, 18, 33, 32, 3, 1), (1, 17, 23, 96, 5, 2),
                                         # grids smaller than the tile count: each workgroup
                                         # walks a run of tiles (window prefetch)
                                         (8, 112, 112, 32, 5, 1), (8, 112, 112, 64, 3, 2)])
def test_dwconv(cuda, n, h, w, c, k, s):
    torch.manual_seed(k * 10 + s)
    x = torch.randn(n, h, w, c, dtype=torch.float64, requires_grad=True)
    wk = torch.randn(k, k, c, dtype=torch.float64)
    if s == 2:
        pt, pb = OE.correct_pad(h, k)
        pl, pr = OE.correct_pad(w, k)
    else:
        pt, pb, _ = OE.same_pad(h, k, 1)
        pl, pr, _ = OE.same_pad(w, k, 1)
    y_ref = OE.dwconv(x.permute(0, 3, 1, 2), wk, s, (pt, pb, pl, pr)).permute(0, 2, 3, 1)
    dy = torch.randn_like(y_ref)
    y_ref.backward(dy)
    oh, ow = y_ref.shape[1:3]
    y = torch.empty(n, oh, ow, c, device=cuda)
    K.dwconv_fwd(dev(x.detach(), cuda), dev(wk, cuda), k, s, pt, pl, y)
    dx = torch.empty(n, h, w, c, device=cuda)
    K.dwconv_dgrad(dev(dy, cuda), dev(wk, cuda), k, s, pt, pl, dx)
    torch.cuda.synchronize()
    assert rel_err(y, y_ref) < 1e-5
    assert rel_err(dx, x.grad) < 1e-5


@pytest.mark.parametrize("k", [3, 5])
@pytest.mark.parametrize("pt,pl", [(0, 0), (0, 1), (1, 0), (1, 1), (2, 1), (2, 2)])
@pytest.mark.parametrize("h,w", [(9, 11), (10, 7)])
def test_dwconv_dgrad_stride2_every_pad_parity(cuda, k, pt, pl, h, w):
    """The 2x2-block stride-2 dgrad (one kernel per pad parity) against autograd, odd and even
    sizes (ragged last block row / column), with accumulate."""
    if pt >= k or pl >= k:
        pytest.skip("pad >= kernel")
    n, c = 2, 8
    torch.manual_seed(k * 100 + pt * 10 + pl)
    x = torch.randn(n, h, w, c, dtype=torch.float64, requires_grad=True)
    wk = torch.randn(k, k, c, dtype=torch.float64)
    oh, ow = (h + pt - k) // 2 + 1, (w + pl - k) // 2 + 1
    pb = max(0, (oh - 1) * 2 + k - h - pt)
    pr = max(0, (ow - 1) * 2 + k - w - pl)
    y_ref = OE.dwconv(x.permute(0, 3, 1, 2), wk, 2, (pt, pb, pl, pr)).permute(0, 2, 3, 1)
    assert y_ref.shape[1:3] == (oh, ow)
    dy = torch.randn_like(y_ref)
    y_ref.backward(dy)
    dx = torch.full((n, h, w, c), 0.5, device=cuda)
    K.dwconv_dgrad(dev(dy, cuda), dev(wk, cuda), k, 2, pt, pl, dx, accumulate=True)
    torch.cuda.synchronize()
    assert rel_err(dx - 0.5, x.grad) < 1e-5, rel_err(dx - 0.5, x.grad)


@pytest.mark.parametrize("k,s", [(3, 1), (5, 2), (5, 1), (3, 2)])
def test_dwconv_fused_bn_swish(cuda, k, s):
    """pld_dwconv_fwd_bn == dwconv(swish(bn(x))) with batch statistics; padding taps read 0
    (TF pads the activated tensor, not the pre-activation one)."""
    n, h, w, c = 2, 11, 14, 24
    torch.manual_seed(40 + k + s)
    x = torch.randn(n, h, w, c, dtype=torch.float64) * 2 + 0.5
    wk = torch.randn(k, k, c, dtype=torch.float64)
    gamma = torch.rand(c, dtype=torch.float64) + 0.5
    beta = torch.randn(c, dtype=torch.float64) * 0.2
    mean = x.mean(dim=(0, 1, 2))
    invstd = 1.0 / torch.sqrt(x.var(dim=(0, 1, 2), unbiased=False) + 1e-3)
    a = (x - mean) * invstd * gamma + beta
    a = a * torch.sigmoid(a)
    if s == 2:
        pt, pb = OE.correct_pad(h, k)
        pl, pr = OE.correct_pad(w, k)
    else:
        pt, pb, _ = OE.same_pad(h, k, 1)
        pl, pr, _ = OE.same_pad(w, k, 1)
    y_ref = OE.dwconv(a.permute(0, 3, 1, 2), wk, s, (pt, pb, pl, pr)).permute(0, 2, 3, 1)
    oh, ow = y_ref.shape[1:3]
    y = torch.empty(n, oh, ow, c, device=cuda)
    bn = tuple(dev(t, cuda) for t in (mean, invstd, gamma, beta))
    K.dwconv_fwd(dev(x, cuda), dev(wk, cuda), k, s, pt, pl, y, bn=bn, act="swish")
    torch.cuda.synchronize()
    assert rel_err(y, y_ref) < 1e-5


@pytest.mark.parametrize("n,h,w,c,cse", [(2, 6, 6, 96, 4), (3, 14, 14, 1152, 48),
                                         (1, 2, 2, 16, 8), (2, 7, 7, 240, 10),
                                         (2, 5, 5, 672, 28)])
def test_se_fwd_bwd(cuda, n, h, w, c, cse):
    torch.manual_seed(c)
    a = torch.randn(n, h, w, c, dtype=torch.float64, requires_grad=True)
    w1 = torch.randn(1, 1, c, cse, dtype=torch.float64) * 0.2
    b1 = torch.randn(cse, dtype=torch.float64) * 0.1
    w2 = torch.randn(1, 1, cse, c, dtype=torch.float64) * 0.2
    b2 = torch.randn(c, dtype=torch.float64) * 0.1
    an = a.permute(0, 3, 1, 2)
    pooled = an.mean(dim=(2, 3), keepdim=True)
    z1 = OE.conv(pooled, w1, b1)
    gate = torch.sigmoid(OE.conv(OE.swish(z1), w2, b2))
    y_ref = (an * gate).permute(0, 2, 3, 1)
    dy = torch.randn_like(y_ref)
    y_ref.backward(dy)
    ga = dev(a.detach(), cuda)
    gp, gz, gg = (torch.empty(n, c, device=cuda), torch.empty(n, cse, device=cuda),
                  torch.empty(n, c, device=cuda))
    K.se_fwd(ga, dev(w1.view(c, cse), cuda), dev(b1, cuda), dev(w2.view(cse, c), cuda),
             dev(b2, cuda), gp, gz, gg)
    torch.cuda.synchronize()
    assert rel_err(gg, gate.view(n, c)) < 1e-5
    addn = torch.empty(n, c, device=cuda)
    gdy = dev(dy, cuda)
    K.se_bwd(gdy, ga, dev(w1.view(c, cse), cuda), dev(w2.view(cse, c), cuda), gz, gg, addn)
    torch.cuda.synchronize()
    da = gdy * gg.view(n, 1, 1, c) + addn.view(n, 1, 1, c)
    assert rel_err(da, a.grad) < 1e-4


@pytest.mark.parametrize("n,h,w,c,cse", [(2, 7, 9, 96, 4), (3, 14, 14, 240, 10),
                                         (2, 33, 29, 16, 4)])
def test_se_with_bn_prologue(cuda, n, h, w, c, cse):
    """pld_se_{fwd,bwd}_bn (SE squeeze of swish(BN(x)) computed on the fly from the pre-BN x)
    against the fp64 restatement of BN + swish + SE."""
    torch.manual_seed(c + 1)
    x = torch.randn(n, h, w, c, dtype=torch.float64) * 2 + 0.3
    mu = x.mean(dim=(0, 1, 2))
    inv = 1.0 / torch.sqrt(x.var(dim=(0, 1, 2), unbiased=False) + 1e-3)
    gam = torch.rand(c, dtype=torch.float64) + 0.5
    bet = torch.randn(c, dtype=torch.float64) * 0.2
    a = OE.swish((x - mu) * inv * gam + bet).detach().requires_grad_(True)
    w1 = torch.randn(1, 1, c, cse, dtype=torch.float64) * 0.2
    b1 = torch.randn(cse, dtype=torch.float64) * 0.1
    w2 = torch.randn(1, 1, cse, c, dtype=torch.float64) * 0.2
    b2 = torch.randn(c, dtype=torch.float64) * 0.1
    an = a.permute(0, 3, 1, 2)
    gate = torch.sigmoid(OE.conv(OE.swish(OE.conv(an.mean(dim=(2, 3), keepdim=True), w1, b1)),
                                 w2, b2))
    y_ref = (an * gate).permute(0, 2, 3, 1)
    dy = torch.randn_like(y_ref)
    y_ref.backward(dy)
    bn = tuple(dev(t, cuda) for t in (mu, inv, gam, bet))
    gx = dev(x, cuda)
    gp, gz, gg = (torch.empty(n, c, device=cuda), torch.empty(n, cse, device=cuda),
                  torch.empty(n, c, device=cuda))
    W1, W2 = dev(w1.view(c, cse), cuda), dev(w2.view(cse, c), cuda)
    K.se_fwd(gx, W1, dev(b1, cuda), W2, dev(b2, cuda), gp, gz, gg, bn=bn, act="swish")
    torch.cuda.synchronize()
    assert rel_err(gg, gate.view(n, c)) < 1e-5
    addn = torch.empty(n, c, device=cuda)
    gdy = dev(dy, cuda)
    K.se_bwd(gdy, gx, W1, W2, gz, gg, addn, bn=bn, act="swish")
    torch.cuda.synchronize()
    da = gdy * gg.view(n, 1, 1, c) + addn.view(n, 1, 1, c)
    assert rel_err(da, a.grad) < 1e-4
    # the SE backward with the block BN's backward folded into its squeeze sweep
    # (pld_se_bwd_bn_full) == pld_se_bwd_bn + pld_bn_bwd(gate, addn)
    gam_d, bet_d = bn[2], bn[3]
    dx_ref = torch.empty_like(gx)
    dg_ref, db_ref = torch.empty(c, device=cuda), torch.empty(c, device=cuda)
    K.bn_bwd(gx, gdy, n * h * w, c, bn[0], bn[1], gam_d, bet_d, "swish", dx_ref, dg_ref, db_ref,
             gate=gg, addn=addn, hw=h * w)
    addn2, dx2 = torch.empty_like(addn), torch.empty_like(gx)
    dg2, db2 = torch.empty(c, device=cuda), torch.empty(c, device=cuda)
    K.se_bwd_bn_full(gdy, gx, bn, W1, W2, gz, gg, addn2, dx2, dg2, db2, act="swish")
    torch.cuda.synchronize()
    assert rel_err(addn2, addn) < 1e-6
    assert rel_err(dg2, dg_ref) < 1e-5 and rel_err(db2, db_ref) < 1e-5
    assert rel_err(dx2, dx_ref) < 1e-5, rel_err(dx2, dx_ref)


# ------------------------------------------------------------------------------- sampler
@pytest.mark.parametrize("ci", range(4))
@pytest.mark.parametrize("strategy", ["thresh", "info", "pure", "masked"])
def test_sampler_bit_exact_vs_oracle(cuda, golden, ci, strategy):
    h, w, L, R = [int(v) for v in golden[f"c{ci}_shape"]]
    mask = np.unpackbits(golden[f"c{ci}_mask"])[: h * w].reshape(h, w).astype(np.float32)
    gt = golden[f"c{ci}_codes"].astype(np.float32) / np.float32(255)
    draws = golden[f"c{ci}_{strategy}_draws"].astype(np.int32)
    ref, _ = S.sample_masked_point_batch(strategy, mask, gt, R, L, draws)
    B = 2  # two copies of the image: per-image indexing
    gmask = dev(torch.from_numpy(np.stack([mask, mask])), cuda)
    ggt = dev(torch.from_numpy(np.stack([gt, gt])), cuda)
    vi = torch.empty(B, h * w, dtype=torch.int32, device=cuda)
    nv = torch.empty(B, dtype=torch.int32, device=cuda)
    mm = torch.empty(B, 2, device=cuda)
    K.sampler_compact(gmask, ggt, vi, nv, mm)
    gd = torch.from_numpy(np.stack([draws, draws])).to(cuda).contiguous()
    out = torch.empty((B,) + ref.shape, device=cuda)
    K.sampler_rank(ggt, vi, nv, mm, gd, R, L, strategy, out)
    torch.cuda.synchronize()
    assert nv.cpu().tolist() == [int(mask.sum())] * 2
    for b in range(B):
        np.testing.assert_array_equal(out[b].cpu().numpy(), ref)


@pytest.mark.parametrize("L,R", [(64, 1000), (20, 300), (9, 250), (64, 30)])
@pytest.mark.parametrize("strategy", ["info", "thresh", "masked", "pure"])
def test_sampler_stress_shapes_bit_exact(cuda, L, R, strategy):
    """BASELINE cfg5 (448x448, L=64, R=1000: 5,000 Info candidates per image -> the wave-per-list
    candidate kernel and the chunked top-R selection) and ragged L against the oracle, on 8-bit
    depth codes (many tied depths and tied scores)."""
    h, w, B = 448, 448, 2
    rng = np.random.default_rng(L * 1000 + R)
    gts = (np.round(rng.random((B, h, w)) * 255) / 255).astype(np.float32)
    masks = (rng.random((B, h, w)) < 0.9).astype(np.float32)
    nc = {"info": 5 * R, "thresh": int(R * 1.5), "masked": int(R * 1.5), "pure": int(R * 0.8)}
    draws = np.stack([rng.integers(0, int(masks[b].sum()), (nc[strategy], L)) for b in range(B)])
    draws = draws.astype(np.int32)
    vi = torch.empty(B, h * w, dtype=torch.int32, device=cuda)
    nv = torch.empty(B, dtype=torch.int32, device=cuda)
    mm = torch.empty(B, 2, device=cuda)
    ggt = dev(torch.from_numpy(gts), cuda)
    K.sampler_compact(dev(torch.from_numpy(masks), cuda), ggt, vi, nv, mm)
    refs = [S.sample_masked_point_batch(strategy, masks[b], gts[b], R, L, draws[b].reshape(-1))[0]
            for b in range(B)]
    out = torch.empty((B,) + refs[0].shape, device=cuda)
    K.sampler_rank(ggt, vi, nv, mm, torch.from_numpy(draws).to(cuda).contiguous(), R, L,
                   strategy, out)
    torch.cuda.synchronize()
    for b in range(B):
        np.testing.assert_array_equal(out[b].cpu().numpy(), refs[b])


@pytest.mark.parametrize("h,w", [(448, 448), (37, 53), (1, 5), (130, 129)])
def test_sampler_compact_matches_np_where(cuda, h, w):
    """Valid-pixel lists == np.where(mask > 0) order (sampling.py:135), nvalid, whole-image gt
    min/max; images cover the empty mask, the full mask and ragged multi-segment sizes."""
    rng = np.random.default_rng(h * 1000 + w)
    B = 4
    mask = (rng.random((B, h, w)) < 0.9).astype(np.float32)
    mask[1] = 0.0
    mask[2] = 1.0
    gt = rng.random((B, h, w)).astype(np.float32)
    gm, gg = dev(torch.from_numpy(mask), cuda), dev(torch.from_numpy(gt), cuda)
    vi = torch.full((B, h * w), -7, dtype=torch.int32, device=cuda)
    nv = torch.empty(B, dtype=torch.int32, device=cuda)
    mm = torch.empty(B, 2, device=cuda)
    K.sampler_compact(gm, gg, vi, nv, mm)
    torch.cuda.synchronize()
    for b in range(B):
        ref = np.flatnonzero(mask[b].reshape(-1) > 0)
        assert int(nv[b]) == ref.size
        np.testing.assert_array_equal(vi[b, :ref.size].cpu().numpy(), ref)
        assert float(mm[b, 0]) == gt[b].min() and float(mm[b, 1]) == gt[b].max()


def test_sampler_draws_uniform_and_in_range(cuda):
    B, n_cand, L = 4, 500, 5
    nv = torch.tensor([1, 7, 1000, 200000], dtype=torch.int32, device=cuda)
    d = torch.empty(B, n_cand, L, dtype=torch.int32, device=cuda)
    K.sampler_draw(nv, n_cand, L, seed=1234, step=7, image_offset=0, draws=d)
    d2 = torch.empty_like(d)
    K.sampler_draw(nv, n_cand, L, seed=1234, step=7, image_offset=0, draws=d2)
    d3 = torch.empty_like(d)
    K.sampler_draw(nv, n_cand, L, seed=1234, step=8, image_offset=0, draws=d3)
    torch.cuda.synchronize()
    d, d2, d3 = d.cpu(), d2.cpu(), d3.cpu()
    assert torch.equal(d, d2) and not torch.equal(d, d3)
    for b, n in enumerate([1, 7, 1000, 200000]):
        assert int(d[b].min()) >= 0 and int(d[b].max()) < n
    counts = torch.bincount(d[1].flatten(), minlength=7).double()
    exp = n_cand * L / 7
    assert float(((counts - exp) ** 2 / exp).sum()) < 30  # chi2, 6 dof
    # image_offset makes draws independent of the shard layout
    e = torch.empty(2, n_cand, L, dtype=torch.int32, device=cuda)
    K.sampler_draw(nv[2:].contiguous(), n_cand, L, seed=1234, step=7, image_offset=2, draws=e)
    assert torch.equal(e.cpu(), d[2:])


# ------------------------------------------------------------------- ResNet / ReDWeb pieces
@pytest.mark.parametrize("case", [(2, 8, 8, 64, 256, 2), (1, 14, 10, 256, 128, 2),
                                  (2, 7, 9, 32, 20, 2), (1, 6, 6, 16, 64, 3)])
@pytest.mark.parametrize("math", MATHS)
def test_strided_1x1_conv_fwd_dgrad_wgrad(cuda, case, math):
    """ResNet-50 downsampling / projection convs: 1x1, stride s, no padding (keras resnet
    block1 `_0_conv` / `_1_conv`), including odd sizes where the last row/col is skipped."""
    n, h, w, cin, cout, s = case
    torch.manual_seed(11)
    x = torch.randn(n, h, w, cin, dtype=torch.float64)
    wt = torch.randn(1, 1, cin, cout, dtype=torch.float64) / np.sqrt(cin)
    b = torch.randn(cout, dtype=torch.float64)
    xr, wr = x.clone().requires_grad_(True), wt.clone().requires_grad_(True)
    y_ref = OE.conv(xr.permute(0, 3, 1, 2), wr, b, s).permute(0, 2, 3, 1)
    oh, ow = y_ref.shape[1], y_ref.shape[2]
    dy = torch.randn_like(y_ref)
    y_ref.backward(dy)
    gx, gw = dev(x, cuda), dev(wt, cuda)
    args = K.conv_args(gx, None, 1, 1, s, 0, 0, oh, ow, cout, math=math)
    tol = CONV_TOL[math]
    y = torch.empty(n, oh, ow, cout, device=cuda)
    K.conv2d_fwd(args, K.filter_to_native(gw), dev(b, cuda), y)
    gdy = dev(dy, cuda)
    dw = torch.empty(1, 1, cin, cout, device=cuda)
    K.conv2d_wgrad(args, gdy, dw)
    dx = torch.full_like(gx, 3.0)
    K.conv2d_dgrad(args, gdy, K.filter_to_dgrad(gw), dx, acc1=True)
    torch.cuda.synchronize()
    assert rel_err(y, y_ref) < tol
    assert rel_err(dw, wr.grad) < tol
    assert rel_err(dx - 3.0, xr.grad) < tol
    dx2 = torch.empty_like(gx)
    K.conv2d_dgrad(args, gdy, K.filter_to_dgrad(gw), dx2)
    torch.cuda.synchronize()
    assert rel_err(dx2, xr.grad) < tol


def test_resnet_stem_conv(cuda):
    """ZeroPadding2D(3) + Conv2D(64, 7, strides=2) (+bias) on a 3-channel image."""
    n, h, w = 2, 32, 40
    torch.manual_seed(12)
    x = torch.randn(n, h, w, 3, dtype=torch.float64) * 50
    wt = torch.randn(7, 7, 3, 64, dtype=torch.float64) * 0.05
    b = torch.randn(64, dtype=torch.float64)
    y_ref = OE.conv(x.permute(0, 3, 1, 2), wt, b, 2, (3, 3, 3, 3)).permute(0, 2, 3, 1)
    oh, ow = y_ref.shape[1:3]
    assert (oh, ow) == (h // 2, w // 2)
    args = K.conv_args(dev(x, cuda), None, 7, 7, 2, 3, 3, oh, ow, 64)
    y = torch.empty(n, oh, ow, 64, device=cuda)
    K.conv2d_fwd(args, K.filter_to_native(dev(wt, cuda)), dev(b, cuda), y)
    torch.cuda.synchronize()
    assert rel_err(y, y_ref) < 1e-5


@pytest.mark.parametrize("shape,relu", [((2, 16, 20, 64), True), ((1, 9, 7, 12), False),
                                        ((2, 15, 15, 5), True)])
def test_maxpool_zero_padded(cuda, shape, relu):
    from oracle import redweb as OR
    torch.manual_seed(13)
    x = torch.randn(*shape, dtype=torch.float64).float().double()  # fp32-exact: same order
    if relu:
        x = torch.relu(x)  # zeros tie with the padding, as after conv1_relu
    xr = x.clone().requires_grad_(True)
    y_ref = OR.maxpool_zero_padded(xr.permute(0, 3, 1, 2)).permute(0, 2, 3, 1)
    dy = torch.randn_like(y_ref)
    y_ref.backward(dy)
    n, h, w, c = shape
    oh, ow = y_ref.shape[1:3]
    y = torch.empty(n, oh, ow, c, device=cuda)
    am = torch.empty(n, oh, ow, c, dtype=torch.uint8, device=cuda)
    K.maxpool2d_fwd(dev(x, cuda), 3, 2, 1, 1, y, am)
    dx = torch.empty(n, h, w, c, device=cuda)
    K.maxpool2d_bwd(dev(dy, cuda), am, 3, 2, 1, 1, dx)
    torch.cuda.synchronize()
    assert rel_err(y, y_ref) == 0.0
    assert rel_err(dx, xr.grad) < 1e-6
    dx.fill_(0.5)
    K.maxpool2d_bwd(dev(dy, cuda), am, 3, 2, 1, 1, dx, accumulate=True)
    torch.cuda.synchronize()
    assert rel_err(dx - 0.5, xr.grad) < 1e-6


@pytest.mark.parametrize("dres_acc", [True, False])
@pytest.mark.parametrize("rows,c,act", [(3000, 64, "relu"), (517, 256, "none"),
                                        (200, 6, "relu"), (4099, 128, "relu")])
def test_bn_add_forward_backward(cuda, rows, c, act, dres_acc):
    """pld_bn_add_apply / pld_bn_add_bwd vs autograd; a fresh dres with an activation takes the
    dz-storing reduction pass (the elementwise pass then reads (x, dz))."""
    from oracle import redweb as OR
    torch.manual_seed(rows + c)
    x = torch.randn(rows, c, dtype=torch.float64) * 2 + 0.5
    res = torch.randn(rows, c, dtype=torch.float64)
    gamma = torch.rand(c, dtype=torch.float64) + 0.5
    beta = torch.randn(c, dtype=torch.float64)
    xr, rr, gr, br = (t.clone().requires_grad_(True) for t in (x, res, gamma, beta))
    z = OR.bn_train(xr.T.reshape(1, c, rows, 1), gr, br, OR.RESNET_BN_EPS)
    z = z.reshape(c, rows).T + rr
    y_ref = torch.relu(z) if act == "relu" else z
    dy = torch.randn_like(y_ref)
    y_ref.backward(dy)
    gx = dev(x, cuda)
    gm, gi = torch.empty(c, device=cuda), torch.empty(c, device=cuda)
    K.bn_stats(gx, rows, c, gm, gi, None, None, OR.RESNET_BN_EPS)
    y = torch.empty_like(gx)
    gres, ggam, gbet = dev(res, cuda), dev(gamma, cuda), dev(beta, cuda)
    K.bn_add_apply(gx, rows, c, gm, gi, ggam, gbet, gres, act, y)
    dx = torch.empty_like(gx)
    base = 2.0 if dres_acc else 0.0
    dres = torch.full_like(gx, 2.0)
    dg, db = torch.empty(c, device=cuda), torch.empty(c, device=cuda)
    K.bn_add_bwd(gx, dev(dy, cuda), rows, c, gm, gi, ggam, gbet, gres, act, dx, dres, dg, db,
                 dres_accumulate=dres_acc)
    torch.cuda.synchronize()
    assert rel_err(y, y_ref) < 1e-5
    assert rel_err(dx, xr.grad) < 1e-4
    assert rel_err(dres - base, rr.grad) < 1e-5
    assert rel_err(dg, gr.grad) < 1e-5
    assert rel_err(db, br.grad) < 1e-5


@pytest.mark.parametrize("n,hw,c", [(4, 49, 40), (3, 25, 6), (2, 196, 112), (5, 9, 3)])
def test_bn_scale_add_fused_matches_unfused(cuda, n, hw, c):
    """The EfficientNet residual block output (project BN, drop-connect scale, residual add) in
    one pass (pld_bn_scale_add_apply) and its BN backward with the scale folded in
    (pld_bn_bwd_scaled) are bit-identical to bn_apply + residual_add and scale_per_sample +
    bn_bwd; the float4 (c % 4 == 0) and scalar paths, the row-blocked and general reductions."""
    torch.manual_seed(n * 1000 + hw + c)
    rows = n * hw
    x = dev(torch.randn(rows, c) * 2 + 0.5, cuda)
    res = dev(torch.randn(rows, c), cuda)
    dy = dev(torch.randn(rows, c), cuda)
    gam = dev(torch.rand(c) + 0.5, cuda)
    bet = dev(torch.randn(c), cuda)
    sc = dev(torch.tensor([0.0, 1.25, 1.25, 1.25, 0.0][:n]), cuda)
    gm, gi = torch.empty(c, device=cuda), torch.empty(c, device=cuda)
    K.bn_stats(x, rows, c, gm, gi)
    y_un = torch.empty_like(x)
    K.bn_apply(x, rows, c, gm, gi, gam, bet, "none", y_un)
    K.residual_add(y_un.view(n, hw, c), sc, res.view(n, hw, c), y_un.view(n, hw, c))
    y = torch.empty_like(x)
    K.bn_scale_add_apply(x, rows, c, gm, gi, gam, bet, sc, hw, res, "none", y)
    ds = torch.empty_like(x)
    K.scale_per_sample(dy.view(n, hw, c), sc, ds.view(n, hw, c))
    dx_un, dg_un, db_un = torch.empty_like(x), torch.empty(c, device=cuda), torch.empty(c, device=cuda)
    K.bn_bwd(x, ds, rows, c, gm, gi, gam, bet, "none", dx_un, dg_un, db_un)
    dx, dg, db = torch.full_like(x, 7.0), torch.empty(c, device=cuda), torch.empty(c, device=cuda)
    K.bn_bwd_scaled(x, dy, rows, c, gm, gi, gam, bet, "none", sc, hw, dx, dg, db)
    torch.cuda.synchronize()
    assert torch.equal(y, y_un)
    # ... and to the reference's two-step fp32 form: Dropout's product rounded, then Add's sum
    y_bn = torch.empty_like(x)
    K.bn_apply(x, rows, c, gm, gi, gam, bet, "none", y_bn)
    two_step = y_bn.view(n, hw, c) * sc.view(n, 1, 1) + res.view(n, hw, c)
    torch.cuda.synchronize()
    assert torch.equal(y.view(n, hw, c), two_step)
    assert torch.equal(dx, dx_un)
    assert torch.equal(dg, dg_un) and torch.equal(db, db_un)
    # a dropped image passes only its residual
    assert torch.equal(y.view(n, hw, c)[0], res.view(n, hw, c)[0])


# thin 1x1 convs (csrc/thin.hip): K <= 48, VALU with the filter in SGPRs; ragged
# 64-row tails, every K instance, CH 8 and 16 column chunks, accumulate, fwd bias
@pytest.mark.parametrize("n,h,w,cin,cout", [(2, 7, 9, 16, 96), (1, 11, 13, 24, 144),
                                            (1, 5, 5, 40, 96), (2, 9, 9, 96, 24),
                                            (1, 6, 7, 144, 24), (3, 5, 5, 32, 16),
                                            (1, 8, 8, 8, 40), (1, 3, 3, 48, 64),
                                            (1, 64, 64, 64, 8)])
def test_thin_1x1_conv(cuda, n, h, w, cin, cout):
    torch.manual_seed(cin * 1000 + cout)
    x = torch.randn(n, h, w, cin, dtype=torch.float64)
    wt = torch.randn(1, 1, cin, cout, dtype=torch.float64) / np.sqrt(cin)
    b = torch.randn(cout, dtype=torch.float64)
    y_ref = torch.einsum("nhwc,cd->nhwd", x, wt[0, 0]) + b
    dy = torch.randn(n, h, w, cout, dtype=torch.float64)
    dx_ref = torch.einsum("nhwd,cd->nhwc", dy, wt[0, 0])
    gx, gw = dev(x, cuda), dev(wt, cuda)
    args = K.conv_args(gx, None, 1, 1, 1, 0, 0, h, w, cout, math="fp32")
    lib = _lib.lib()
    thin_fwd = cin % 8 == 0 and cin <= 48 and cout % 8 == 0 and cin * cout <= 4096
    thin_dg = cout % 8 == 0 and cout <= 48 and cin % 8 == 0 and cin * cout <= 4096
    assert thin_fwd or thin_dg
    # PLD_KIND_DIRECT (2) = the thin path
    assert (lib.pld_conv_kernel_kind(C.byref(args), 0) == 2) == thin_fwd
    assert (lib.pld_conv_kernel_kind(C.byref(args), 1) == 2) == thin_dg
    y = torch.empty(n, h, w, cout, device=cuda)
    K.conv2d_fwd(args, K.filter_to_native(gw), dev(b, cuda), y)
    torch.cuda.synchronize()
    assert rel_err(y, y_ref) < 1e-5, rel_err(y, y_ref)
    K.conv2d_fwd(args, K.filter_to_native(gw), dev(b, cuda), y, accumulate=True)
    torch.cuda.synchronize()
    assert rel_err(y, 2 * y_ref) < 1e-5
    dx = torch.full_like(gx, 0.25)
    K.conv2d_dgrad(args, dev(dy, cuda), K.filter_to_dgrad(gw), dx, None, acc1=True)
    torch.cuda.synchronize()
    assert rel_err(dx - 0.25, dx_ref) < 1e-5, rel_err(dx - 0.25, dx_ref)


# ------------------------------------------------- fused BN+ReLU -> upsample x2 -> 3x3 conv to 1
@pytest.mark.parametrize("n,h,w,c", [(2, 5, 7, 8), (1, 16, 16, 32), (2, 33, 20, 32),
                                     (2, 224, 224, 32)])
def test_upconv_matches_unfused_path(cuda, n, h, w, c):
    """pld_upconv_{fwd,wgrad,dgrad,bwd} (csrc/upconv.hip: the 9 tap maps at 1x resolution)
    against the unfused kernels they replace: pld_upsample2x_fwd_bn + pld_conv2d_fwd / _wgrad /
    _dgrad + pld_upsample2x_bwd, then pld_bn_bwd (relu) for the fused BN backward."""
    g = torch.Generator(device=cuda).manual_seed(n * h + w)
    x = torch.randn(n, h, w, c, device=cuda, generator=g)
    mean = torch.randn(c, device=cuda, generator=g) * 0.1
    invstd = torch.rand(c, device=cuda, generator=g) + 0.5
    gamma = torch.rand(c, device=cuda, generator=g) + 0.5
    beta = torch.randn(c, device=cuda, generator=g) * 0.1
    bn = (mean, invstd, gamma, beta)
    wt = torch.randn(3, 3, c, 1, device=cuda, generator=g) / (9 * c) ** 0.5
    bias = torch.randn(1, device=cuda, generator=g)
    dy = torch.randn(n, 2 * h, 2 * w, 1, device=cuda, generator=g)
    # unfused reference
    up = torch.empty(n, 2 * h, 2 * w, c, device=cuda)
    K.upsample2x_fwd(x, up, bn=bn, act="relu")
    args = K.conv_args(up, None, 3, 3, 1, 1, 1, 2 * h, 2 * w, 1, math="fp32")
    wn, wd = K.filter_to_native(wt), K.filter_to_dgrad(wt)
    y_ref = torch.empty(n, 2 * h, 2 * w, 1, device=cuda)
    K.conv2d_fwd(args, wn, bias, y_ref)
    dw_ref = torch.empty_like(wt)
    K.conv2d_wgrad(args, dy, dw_ref)
    dup = torch.empty_like(up)
    K.conv2d_dgrad(args, dy, wd, dup)
    dact_ref = torch.empty_like(x)
    K.upsample2x_bwd(dup, dact_ref)
    # fused
    y = torch.empty_like(y_ref)
    K.upconv_fwd(x, bn, wn, bias, y)
    dw = torch.empty_like(wt)
    K.upconv_wgrad(x, bn, dy, dw)
    dact = torch.empty_like(x)
    K.upconv_dgrad(dy, wt, dact)
    # the one-pass backward with the BN + ReLU backward folded in
    dact2, dw2, dx2 = torch.empty_like(x), torch.empty_like(wt), torch.empty_like(x)
    dg2, db2 = torch.empty(c, device=cuda), torch.empty(c, device=cuda)
    K.upconv_bwd(x, bn, wn, dy, dact2, dw=dw2, dx=dx2, dgamma=dg2, dbeta=db2)
    dx_ref = torch.empty_like(x)
    dg_ref, db_ref = torch.empty(c, device=cuda), torch.empty(c, device=cuda)
    K.bn_bwd(x, dact_ref, n * h * w, c, mean, invstd, gamma, beta, "relu", dx_ref, dg_ref,
             db_ref)
    torch.cuda.synchronize()
    assert rel_err(y, y_ref) < 1e-5
    assert rel_err(dw, dw_ref) < 1e-5
    assert rel_err(dact, dact_ref) < 1e-5
    assert torch.equal(dact2, dact) and torch.equal(dw2, dw)
    assert rel_err(dx2, dx_ref) < 1e-4, rel_err(dx2, dx_ref)
    assert rel_err(dg2, dg_ref) < 1e-5 and rel_err(db2, db_ref) < 1e-5
    # and against torch-CPU fp64 for the whole composition
    x64 = x.double().cpu().permute(0, 3, 1, 2)
    a = torch.relu((x64 - mean.double().cpu().view(1, -1, 1, 1)) *
                   invstd.double().cpu().view(1, -1, 1, 1) * gamma.double().cpu().view(1, -1, 1, 1)
                   + beta.double().cpu().view(1, -1, 1, 1)).requires_grad_(True)
    u = F.interpolate(a, scale_factor=2, mode="bilinear", align_corners=False)
    w64 = wt.double().cpu().permute(3, 2, 0, 1).contiguous().requires_grad_(True)
    o = F.conv2d(u, w64, bias.double().cpu(), padding=1)
    o.backward(dy.double().cpu().permute(0, 3, 1, 2))
    assert rel_err(y, o.detach().permute(0, 2, 3, 1)) < 1e-5
    assert rel_err(dw, w64.grad.permute(2, 3, 1, 0)) < 1e-5
    assert rel_err(dact, a.grad.permute(0, 2, 3, 1)) < 1e-5


# --------------------------------------- thin-N 1x1 convs with the neighbouring BN folded in
@pytest.mark.parametrize("n,hw,k,cout,gate", [(2, 100, 96, 24, True), (3, 57, 144, 40, True),
                                              (2, 64, 32, 16, False), (1, 300, 240, 40, True),
                                              (2, 33, 144, 24, False)])
def test_pgemm_bn_act_and_bn_bwd(cuda, n, hw, k, cout, gate):
    """pld_pgemm_bn_act == pld_bn_apply(swish, gate) + exact-fp32 1x1 conv, and
    pld_bn_bwd_coeffs + pld_pgemm_bn_bwd == pld_bn_bwd(swish) + exact-fp32 1x1 dgrad
    (csrc/pgemm.hip; ragged row counts, every N width class)."""
    g = torch.Generator(device=cuda).manual_seed(k + cout + hw)
    rows = n * hw
    x = torch.randn(n, hw, 1, k, device=cuda, generator=g) * 1.5 + 0.2
    mean = torch.randn(k, device=cuda, generator=g) * 0.1
    invstd = torch.rand(k, device=cuda, generator=g) + 0.5
    gamma = torch.rand(k, device=cuda, generator=g) + 0.5
    beta = torch.randn(k, device=cuda, generator=g) * 0.1
    gt = torch.rand(n, k, device=cuda, generator=g) if gate else None
    wt = torch.randn(1, 1, k, cout, device=cuda, generator=g) / k ** 0.5
    wn = K.filter_to_native(wt)                      # [cout][k]
    # forward: reference = apply then conv (fp32 math)
    a = torch.empty_like(x)
    K.bn_apply(x, rows, k, mean, invstd, gamma, beta, "swish", a, gate=gt, hw=hw)
    y_ref = torch.empty(n, hw, 1, cout, device=cuda)
    K.conv2d_fwd(K.conv_args(a, None, 1, 1, 1, 0, 0, hw, 1, cout, math="fp32"), wn, None, y_ref)
    y = torch.empty_like(y_ref)
    K.pgemm_bn_act(x, rows, k, mean, invstd, gamma, beta, "swish", wn, cout, y, gate=gt, hw=hw)
    # backward: the expand-dgrad form (w = the dgrad filter [cin][cexp] of a cin -> cexp conv)
    cin = cout
    w2 = torch.randn(1, 1, cin, k, device=cuda, generator=g) / k ** 0.5
    wd = K.filter_to_dgrad(w2)                       # [cin][k]
    dy = torch.randn_like(x)
    dx_ref = torch.empty_like(x)
    dg_ref, db_ref = torch.empty(k, device=cuda), torch.empty(k, device=cuda)
    K.bn_bwd(x, dy, rows, k, mean, invstd, gamma, beta, "swish", dx_ref, dg_ref, db_ref)
    gx_ref = torch.empty(n, hw, 1, cin, device=cuda)
    K.conv2d_dgrad(K.conv_args(gx_ref, None, 1, 1, 1, 0, 0, hw, 1, k, math="fp32"), dx_ref, wd,
                   gx_ref)
    k12 = torch.empty(2 * k, device=cuda)
    dg, db = torch.empty(k, device=cuda), torch.empty(k, device=cuda)
    K.bn_bwd_coeffs(x, dy, rows, k, mean, invstd, gamma, beta, "swish", dg, db, k12)
    gx = torch.empty_like(gx_ref)
    K.pgemm_bn_bwd(x, dy, rows, k, mean, invstd, gamma, beta, "swish", k12, wd, cin, gx)
    torch.cuda.synchronize()
    assert rel_err(y, y_ref) < 1e-5, rel_err(y, y_ref)
    assert torch.equal(dg, dg_ref) and torch.equal(db, db_ref)
    assert rel_err(gx, gx_ref) < 1e-5, rel_err(gx, gx_ref)
    # accumulate form
    K.pgemm_bn_act(x, rows, k, mean, invstd, gamma, beta, "swish", wn, cout, y, gate=gt, hw=hw,
                   accumulate=True)
    torch.cuda.synchronize()
    assert rel_err(y, 2 * y_ref) < 1e-5


@pytest.mark.parametrize("n,h,w,cin,cout", [(2, 20, 17, 16, 96), (3, 8, 8, 24, 144),
                                            (2, 9, 7, 40, 240), (1, 5, 6, 48, 64)])
def test_conv_fwd_bn_stats(cuda, n, h, w, cin, cout):
    """pld_conv2d_fwd_bn_stats (BN statistics gathered in the thin 1x1 kernel's epilogue, or
    conv + pld_bn_stats where the kernel cannot) == pld_conv2d_fwd + pld_bn_stats."""
    g = torch.Generator(device=cuda).manual_seed(cin * cout + h)
    x = torch.randn(n, h, w, cin, device=cuda, generator=g)
    wt = torch.randn(1, 1, cin, cout, device=cuda, generator=g) / cin ** 0.5
    wn = K.filter_to_native(wt)
    rows = n * h * w
    args = K.conv_args(x, None, 1, 1, 1, 0, 0, h, w, cout, math="fp32")
    y_ref = torch.empty(n, h, w, cout, device=cuda)
    K.conv2d_fwd(args, wn, None, y_ref)
    m_ref, i_ref = torch.empty(cout, device=cuda), torch.empty(cout, device=cuda)
    mm_ref, mv_ref = torch.zeros(cout, device=cuda), torch.ones(cout, device=cuda)
    K.bn_stats(y_ref, rows, cout, m_ref, i_ref, mm_ref, mv_ref)
    y = torch.empty_like(y_ref)
    m, i = torch.empty(cout, device=cuda), torch.empty(cout, device=cuda)
    mm, mv = torch.zeros(cout, device=cuda), torch.ones(cout, device=cuda)
    K.conv2d_fwd_bn_stats(args, wn, None, y, m, i, mm, mv)
    torch.cuda.synchronize()
    assert torch.equal(y, y_ref)
    for a, b in ((m, m_ref), (i, i_ref), (mm, mm_ref), (mv, mv_ref)):
        assert rel_err(a, b) < 1e-6, rel_err(a, b)


@pytest.mark.parametrize("n,h,w,c,k,s,pt,pl", [(2, 13, 11, 96, 3, 1, 1, 1),
                                                (1, 9, 10, 40, 5, 1, 2, 2),
                                                (2, 14, 12, 1152, 3, 1, 1, 1),
                                                # the LDS-tiled stride-1 dgrad (c % 16 == 0)
                                                # must match the fused kernel's sums bit for bit
                                                (1, 9, 10, 48, 5, 1, 2, 2),
                                                (4, 28, 28, 672, 5, 1, 2, 2),
                                                (2, 15, 13, 144, 3, 2, 1, 1),
                                                (1, 12, 14, 240, 5, 2, 1, 2)])
def test_dwconv_dgrad_bn_bwd(cuda, n, h, w, c, k, s, pt, pl):
    """The depthwise dgrad with the producing BN + swish's backward fused into its epilogue ==
    pld_dwconv_dgrad then pld_bn_bwd (dx) / pld_bn_bwd_coeffs (k12), overwrite and accumulate,
    stride 1 and 2 (both pad parities), channel quads beyond one workgroup (c = 1152)."""
    g = torch.Generator(device=cuda).manual_seed(c + k + s)
    oh, ow = (h + s - 1) // s, (w + s - 1) // s
    dy = torch.randn(n, oh, ow, c, device=cuda, generator=g)
    wdw = torch.randn(k, k, c, device=cuda, generator=g) / k
    x = torch.randn(n, h, w, c, device=cuda, generator=g) * 2 + 0.3
    mean = torch.randn(c, device=cuda, generator=g) * 0.2
    invstd = torch.rand(c, device=cuda, generator=g) + 0.5
    gamma = torch.randn(c, device=cuda, generator=g)
    beta = torch.randn(c, device=cuda, generator=g) * 0.1
    bnp = (mean, invstd, gamma, beta)
    rows = n * h * w
    for acc in (False, True):
        pre = torch.randn(n, h, w, c, device=cuda, generator=g)
        dact_ref = pre.clone()
        K.dwconv_dgrad(dy, wdw, k, s, pt, pl, dact_ref, accumulate=acc)
        dx_ref = torch.empty_like(x)
        dg_ref, db_ref = torch.empty(c, device=cuda), torch.empty(c, device=cuda)
        K.bn_bwd(x, dact_ref, rows, c, *bnp, "swish", dx_ref, dg_ref, db_ref)
        k12_ref = torch.empty(2 * c, device=cuda)
        K.bn_bwd_coeffs(x, dact_ref, rows, c, *bnp, "swish", dg_ref.clone(), db_ref.clone(),
                        k12_ref)
        dact = pre.clone()
        dx = torch.empty_like(x)
        dg, db, k12 = torch.empty(c, device=cuda), torch.empty(c, device=cuda), \
            torch.empty(2 * c, device=cuda)
        K.dwconv_dgrad_bn_bwd(dy, wdw, k, s, pt, pl, dact, x, bnp, "swish", dg, db, k12, dx=dx,
                              accumulate=acc)
        torch.cuda.synchronize()
        assert torch.equal(dact, dact_ref)
        for a, r in ((dg, dg_ref), (db, db_ref), (k12, k12_ref)):
            assert rel_err(a, r) < 1e-5, rel_err(a, r)
        assert rel_err(dx, dx_ref) < 1e-5, rel_err(dx, dx_ref)
        # coefficients only (the pgemm_bn_bwd path)
        dact2 = pre.clone()
        K.dwconv_dgrad_bn_bwd(dy, wdw, k, s, pt, pl, dact2, x, bnp, "swish", dg, db, k12,
                              accumulate=acc)
        torch.cuda.synchronize()
        assert torch.equal(dact2, dact_ref) and rel_err(k12, k12_ref) < 1e-5


@pytest.mark.parametrize("math", ["bf16x3", "fp32"])
@pytest.mark.parametrize("n,h,w,cin,c2,k,cout", [(2, 13, 11, 48, 16, 3, 72),
                                                (1, 23, 29, 64, 0, 1, 200),
                                                (3, 9, 10, 96, 0, 3, 40)])
def test_conv_fwd_bn_stats_gemm_epilogue(cuda, math, n, h, w, cin, c2, k, cout):
    """BN statistics from the im2col GEMM epilogue (conv_x3_kernel / conv_igemm_kernel, unsplit
    schedules; split-K schedules take the separate pass) on every schedule: same output, same
    statistics as pld_conv2d_fwd + pld_bn_stats on that schedule. Ragged M tiles (rows % BM),
    ragged N tiles, a concat input and a bias (the statistics are of the stored y)."""
    g = torch.Generator(device=cuda).manual_seed(cin * cout + h + k)
    x = torch.randn(n, h, w, cin, device=cuda, generator=g)
    x2 = torch.randn(n, h, w, c2, device=cuda, generator=g) if c2 else None
    wt = torch.randn(k, k, cin + c2, cout, device=cuda, generator=g) / (k * k * cin) ** 0.5
    b = torch.randn(cout, device=cuda, generator=g) + 0.5
    wn = K.filter_to_native(wt)
    rows = n * h * w
    p = (k - 1) // 2
    n_sched = _lib.lib().pld_conv_num_schedules(K.MATH[math])
    fused = 0
    for t in range(n_sched):
        args = K.conv_args(x, x2, k, k, 1, p, p, h, w, cout, math=math)
        args.tile = t
        y_ref = torch.empty(n, h, w, cout, device=cuda)
        K.conv2d_fwd(args, wn, b, y_ref)
        m_ref, i_ref = torch.empty(cout, device=cuda), torch.empty(cout, device=cuda)
        mm_ref, mv_ref = torch.zeros(cout, device=cuda), torch.ones(cout, device=cuda)
        K.bn_stats(y_ref, rows, cout, m_ref, i_ref, mm_ref, mv_ref)
        y = torch.empty_like(y_ref)
        m, i = torch.empty(cout, device=cuda), torch.empty(cout, device=cuda)
        mm, mv = torch.zeros(cout, device=cuda), torch.ones(cout, device=cuda)
        K.conv2d_fwd_bn_stats(args, wn, b, y, m, i, mm, mv)
        torch.cuda.synchronize()
        assert torch.equal(y, y_ref), t
        for a, r in ((m, m_ref), (i, i_ref), (mm, mm_ref), (mv, mv_ref)):
            assert rel_err(a, r) < 1e-6, (t, rel_err(a, r))
        fused += _lib.lib().pld_conv_schedule_class(K.MATH[math], t) in (0, 3)
    assert fused > 0


@pytest.mark.parametrize("n,h,w,cin,cout", [(2, 20, 17, 40, 240), (1, 13, 11, 112, 672),
                                            (3, 7, 9, 80, 480), (1, 6, 5, 8, 520),
                                            (2, 9, 9, 128, 1152), (1, 3, 7, 56, 200)])
def test_wide1x1(cuda, n, h, w, cin, cout):
    """The streaming bf16x3 1x1 kernel (wide1x1.hip: K <= 128 reductions into wide outputs):
    fwd (+bias, +accumulate), dgrad (the transposed GEMM, +accumulate) and the BN statistics of
    its epilogue against fp64; ragged strips (rows % 32 != 0) and column tiles (N % 32 != 0)."""
    lib = K.lib()
    g = torch.Generator(device=cuda).manual_seed(cin + cout + h)
    x = torch.randn(n, h, w, cin, device=cuda, generator=g)
    wt = torch.randn(1, 1, cin, cout, device=cuda, generator=g) / cin ** 0.5
    b = torch.randn(cout, device=cuda, generator=g)
    wn = K.filter_to_native(wt)
    args = K.conv_args(x, None, 1, 1, 1, 0, 0, h, w, cout, math="bf16x3")
    assert lib.pld_conv_kernel_name(C.byref(args), 0) == b"wide1x1_kernel"
    ref = (x.double().reshape(-1, cin) @ wt.double().reshape(cin, cout) + b.double())
    y = torch.empty(n, h, w, cout, device=cuda)
    K.conv2d_fwd(args, wn, b, y)
    torch.cuda.synchronize()
    assert rel_err(y.reshape(-1, cout), ref) < 2e-5
    K.conv2d_fwd(args, wn, b, y, accumulate=True)
    torch.cuda.synchronize()
    assert rel_err(y.reshape(-1, cout), 2 * ref) < 2e-5
    # BN statistics from the epilogue
    y2 = torch.empty_like(y)
    m, i = torch.empty(cout, device=cuda), torch.empty(cout, device=cuda)
    mm, mv = torch.zeros(cout, device=cuda), torch.ones(cout, device=cuda)
    K.conv2d_fwd_bn_stats(args, wn, None, y2, m, i, mm, mv)
    r2 = x.double().reshape(-1, cin) @ wt.double().reshape(cin, cout)
    torch.cuda.synchronize()
    assert rel_err(y2.reshape(-1, cout), r2) < 2e-5
    m_ref, i_ref = torch.empty(cout, device=cuda), torch.empty(cout, device=cuda)
    K.bn_stats(y2, n * h * w, cout, m_ref, i_ref)
    torch.cuda.synchronize()
    assert rel_err(m, m_ref) < 1e-5 and rel_err(i, i_ref) < 1e-5
    # dgrad of a cout -> cin 1x1 conv runs the same GEMM with K = cout: build it the other way
    dy = torch.randn(n, h, w, cin, device=cuda, generator=g)
    wt2 = torch.randn(1, 1, cout, cin, device=cuda, generator=g) / cin ** 0.5  # fwd cout->cin
    wd = K.filter_to_dgrad(wt2)
    dargs = K.conv_args(torch.empty(n, h, w, cout, device=cuda), None, 1, 1, 1, 0, 0, h, w, cin,
                        math="bf16x3")
    assert lib.pld_conv_kernel_name(C.byref(dargs), 1) == b"wide1x1_kernel"
    dx = torch.full((n, h, w, cout), 0.5, device=cuda)
    K.conv2d_dgrad(dargs, dy, wd, dx, acc1=True)
    dref = dy.double().reshape(-1, cin) @ wt2.double().reshape(cout, cin).t() + 0.5
    torch.cuda.synchronize()
    assert rel_err(dx.reshape(-1, cout), dref) < 2e-5


@pytest.mark.parametrize("n,h,w,c,k,s,pro", [(2, 37, 21, 48, 5, 1, True), (1, 35, 19, 64, 3, 2, True),
                                             (2, 18, 33, 32, 3, 1, False),
                                             (1, 9, 13, 12, 5, 1, True),
                                             (8, 112, 112, 32, 3, 1, True),
                                             (4, 56, 56, 1152, 5, 1, True),
                                             (4, 57, 55, 240, 5, 2, False)])
def test_dwconv_fwd_bn_stats(cuda, n, h, w, c, k, s, pro):
    """pld_dwconv_fwd_bn_stats (the output's BN statistics from the tiled kernel's epilogue; the
    c % 16 != 0 case through the register kernel + pld_bn_stats) == pld_dwconv_fwd_bn +
    pld_bn_stats."""
    g = torch.Generator(device=cuda).manual_seed(c * k + h)
    x = torch.randn(n, h, w, c, device=cuda, generator=g)
    wdw = torch.randn(k, k, c, device=cuda, generator=g) / k
    bn = tuple(torch.rand(c, device=cuda, generator=g) + 0.5 for _ in range(4)) if pro else None
    if s == 1:
        pt = pl = (k - 1) // 2
        oh, ow = h, w
    else:
        pt, pl = k // 2 - 1, k // 2
        oh, ow = (h + 1) // 2, (w + 1) // 2
    y_ref = torch.empty(n, oh, ow, c, device=cuda)
    K.dwconv_fwd(x, wdw, k, s, pt, pl, y_ref, bn=bn, act="swish")
    st_ref = [torch.empty(c, device=cuda), torch.empty(c, device=cuda),
              torch.zeros(c, device=cuda), torch.ones(c, device=cuda)]
    K.bn_stats(y_ref, n * oh * ow, c, *st_ref)
    y = torch.empty_like(y_ref)
    st = [torch.empty(c, device=cuda), torch.empty(c, device=cuda),
          torch.zeros(c, device=cuda), torch.ones(c, device=cuda)]
    K.dwconv_fwd_bn_stats(x, wdw, k, s, pt, pl, y, st, bn=bn, act="swish")
    torch.cuda.synchronize()
    assert torch.equal(y, y_ref)
    for a, b in zip(st, st_ref):
        assert rel_err(a, b) < 1e-6, rel_err(a, b)


@pytest.mark.parametrize("kh,cin,cout", [(3, 1952, 672), (3, 912, 240), (3, 32, 1), (1, 40, 240),
                                         (3, 12, 20), (3, 72, 100)])
def test_filter_refresh(cuda, kh, cin, cout):
    """pld_filter_refresh (tiled transpose + row permutation, splits written beside the fp32
    copies; generic kernels where the shapes are not 8-aligned) == pld_filter_to_native +
    pld_filter_to_dgrad + pld_filter_split, bit for bit."""
    g = torch.Generator(device=cuda).manual_seed(kh * cin + cout)
    w = torch.randn(kh, kh, cin, cout, device=cuda, generator=g)
    nat_ref = K.filter_to_native(w)
    dg_ref = K.filter_to_dgrad(w)
    nat, dg = torch.empty_like(nat_ref), torch.empty_like(dg_ref)
    ns = torch.empty_like(nat_ref) if (kh * kh * cin) % 8 == 0 else None
    ds = torch.empty_like(dg_ref) if (kh * kh * cout) % 8 == 0 else None
    K.filter_refresh(w, nat, ns, dg, ds)
    torch.cuda.synchronize()
    assert torch.equal(nat, nat_ref) and torch.equal(dg, dg_ref)
    if ns is not None:
        assert torch.equal(ns, K.filter_split(nat_ref)) and nat._pld_split is ns
    if ds is not None:
        assert torch.equal(ds, K.filter_split(dg_ref))
    torch.cuda.synchronize()


def test_filter_refresh_batch(cuda):
    """kernels.FilterRefreshBatch (pld_filter_refresh_multi over a device table; the filters
    the batched path does not take keep their own call) == pld_filter_refresh per filter, bit
    for bit: the decoder shapes, a 1x1, one without a dgrad copy, unaligned ones."""
    shapes = [(3, 1952, 672, True), (3, 912, 240, True), (3, 32, 1, True), (1, 40, 240, True),
              (3, 12, 20, True), (3, 72, 100, True), (3, 64, 64, False), (3, 3, 32, True),
              (1, 256, 2048, True)]
    g = torch.Generator(device=cuda).manual_seed(7)
    entries, refs = [], []
    for kh, cin, cout, dgrad in shapes:
        w = torch.randn(kh, kh, cin, cout, device=cuda, generator=g)
        nat = torch.full((cout, kh, kh, cin), -1.0, device=cuda)
        dg = torch.full((cin, kh, kh, cout), -1.0, device=cuda) if dgrad else None
        ns = torch.full_like(nat, -1.0) if (kh * kh * cin) % 8 == 0 else None
        ds = torch.full_like(dg, -1.0) if dgrad and (kh * kh * cout) % 8 == 0 else None
        entries.append((w, nat, ns, dg, ds))
        r = [torch.empty_like(nat), None if ns is None else torch.empty_like(ns),
             None if dg is None else torch.empty_like(dg), None if ds is None else torch.empty_like(ds)]
        K.filter_refresh(w, *r)
        refs.append(r)
    batch = K.FilterRefreshBatch(entries, cuda)
    assert batch.count == 5 and len(batch.single) == 4  # both paths exercised
    batch()
    torch.cuda.synchronize()
    for (w, *got), ref in zip(entries, refs):
        for a, b in zip(got, ref):
            assert (a is None) == (b is None)
            if a is not None:
                assert torch.equal(a, b), w.shape
    # a second call (the per-step form) rewrites the same bytes
    for _, nat, *_ in entries:
        nat.fill_(0.0)
    batch()
    torch.cuda.synchronize()
    for (w, nat, *_), ref in zip(entries, refs):
        assert torch.equal(nat, ref[0])


@pytest.mark.parametrize("n,h,w,pt,pl", [(2, 64, 64, 0, 0), (1, 37, 51, 1, 1), (3, 18, 70, 0, 1),
                                          (1, 448, 448, 0, 0)])
def test_stem3x3(cuda, n, h, w, pt, pl):
    """The direct EfficientNet stem kernel (stem.hip: 3x3 stride 2, 3 -> 32, the Rescaling /
    Normalization prologue on in-image taps, correct_pad's asymmetric zero padding) against
    fp64: plain, +bias, +accumulate, and its epilogue BN statistics against pld_bn_stats of the
    stored output. Ragged 8 x 32 output tiles at the right and bottom edges."""
    g = torch.Generator(device=cuda).manual_seed(h * w + pt)
    oh, ow = (h - 1) // 2 + 1, (w - 1) // 2 + 1
    x = torch.rand(n, h, w, 3, device=cuda, generator=g)
    wt = torch.randn(3, 3, 3, 32, device=cuda, generator=g) / 27 ** 0.5
    b = torch.randn(32, device=cuda, generator=g)
    sc = torch.tensor([1 / 0.229, 1 / 0.224, 1 / 0.225], device=cuda)
    sh = torch.tensor([-0.485 / 0.229, -0.456 / 0.224, -0.406 / 0.225], device=cuda)
    wn = K.filter_to_native(wt)
    args = K.conv_args(x, None, 3, 3, 2, pt, pl, oh, ow, 32, in_scale=sc, in_shift=sh,
                       math="bf16x3")
    assert K.conv_kernel_name(args, "fwd") == "stem3x3_kernel"
    xd = x.double() * sc.double() + sh.double()
    pb = max(0, (oh - 1) * 2 + 3 - h - pt)
    pr = max(0, (ow - 1) * 2 + 3 - w - pl)
    xp = torch.nn.functional.pad(xd.permute(0, 3, 1, 2), (pl, pr, pt, pb))
    ref = torch.nn.functional.conv2d(xp, wt.double().permute(3, 2, 0, 1), stride=2)
    ref = ref.permute(0, 2, 3, 1)[:, :oh, :ow]
    y = torch.empty(n, oh, ow, 32, device=cuda)
    K.conv2d_fwd(args, wn, None, y)
    torch.cuda.synchronize()
    assert rel_err(y, ref) < 1e-6, rel_err(y, ref)
    K.conv2d_fwd(args, wn, b, y, accumulate=True)
    torch.cuda.synchronize()
    assert rel_err(y, 2 * ref + b.double()) < 1e-6
    rows = n * oh * ow
    y2 = torch.empty_like(y)
    m, i = torch.empty(32, device=cuda), torch.empty(32, device=cuda)
    mm, mv = torch.zeros(32, device=cuda), torch.ones(32, device=cuda)
    K.conv2d_fwd_bn_stats(args, wn, b, y2, m, i, mm, mv)
    m_ref, i_ref = torch.empty(32, device=cuda), torch.empty(32, device=cuda)
    mm_ref, mv_ref = torch.zeros(32, device=cuda), torch.ones(32, device=cuda)
    K.bn_stats(y2, rows, 32, m_ref, i_ref, mm_ref, mv_ref)
    torch.cuda.synchronize()
    assert rel_err(y2, ref + b.double()) < 1e-6
    for a, r in ((m, m_ref), (i, i_ref), (mm, mm_ref), (mv, mv_ref)):
        assert rel_err(a, r) < 1e-6, rel_err(a, r)
