"""Thin Python wrappers over the C ABI, taking torch device tensors as memory handles.

PyTorch is plumbing here: tensors provide device memory and the current HIP stream; every
computation is a call into libpldepth_hip.so. Nothing here falls back to torch math.
"""
import contextlib
import ctypes as C
import os

import numpy as np

import torch

from ._lib import ConvArgs, lib

ACT = {"none": 0, "linear": 0, None: 0, "relu": 1, "swish": 2, "sigmoid": 3}
SAMPLER = {"pure": 0, "masked": 1, "thresh": 2, "info": 3}


def ptr(t):
    if t is None:
        return None
    assert t.is_cuda and t.is_contiguous(), "device tensors must be contiguous HIP tensors"
    return C.c_void_p(t.data_ptr())


def stream():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def _f32(t):
    assert t.dtype == torch.float32, t.dtype
    return t


_ws_cache = {}
# workspaces superseded while a captured hipGraph exists: the graph holds their raw pointers,
# so they stay allocated (never returned to the caching allocator) until every graph is gone
_ws_retired = []
_LIVE_GRAPHS = [0]


_WS_SUFFIX = [""]


@contextlib.contextmanager
def workspace_scope(suffix):
    """Every workspace requested inside the block gets its own buffer (key + suffix): calls issued
    on a second stream then never share scratch memory with the same calls on the first."""
    prev = _WS_SUFFIX[0]
    _WS_SUFFIX[0] = prev + suffix
    try:
        yield
    finally:
        _WS_SUFFIX[0] = prev


def workspace(nbytes, key="default"):
    """Reusable byte workspace on the current device (grown on demand, never shrunk)."""
    dev = torch.cuda.current_device()
    k = (dev, key + _WS_SUFFIX[0])
    buf = _ws_cache.get(k)
    if buf is None or buf.numel() < nbytes:
        if buf is not None and _LIVE_GRAPHS[0] > 0:
            _ws_retired.append(buf)
        buf = torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device="cuda")
        _ws_cache[k] = buf
    return buf


# ------------------------------------------------------------------------------------- loss
def listmle_fwd_bwd(pred, y_true, B, R, L, dpred=None, nll=None, loss=None, zero_dpred=True):
    HW = pred.numel() // B
    dpred = torch.empty_like(pred) if dpred is None else dpred
    nll = torch.empty(B * R, dtype=torch.float32, device=pred.device) if nll is None else nll
    loss = torch.empty(1, dtype=torch.float32, device=pred.device) if loss is None else loss
    lib().pld_listmle_fwd_bwd(ptr(_f32(pred)), ptr(_f32(y_true)), B, HW, R, L, ptr(nll),
                              ptr(loss), ptr(dpred), int(zero_dpred), stream())
    return loss, dpred, nll


# ------------------------------------------------------------------------------- optimizer
def adam_amsgrad(param, grad, m, v, vhat, lr, step, beta1=0.9, beta2=0.999, eps=1e-7,
                 grad_scale=1.0):
    lib().pld_adam_amsgrad(ptr(param), ptr(grad), ptr(m), ptr(v), ptr(vhat), param.numel(),
                           float(lr), beta1, beta2, eps, int(step), float(grad_scale), stream())


def adam_amsgrad_dev(param, grad, m, v, vhat, lr_dev, step_dev, beta1=0.9, beta2=0.999,
                     eps=1e-7, grad_scale=1.0):
    lib().pld_adam_amsgrad_dev(ptr(param), ptr(grad), ptr(m), ptr(v), ptr(vhat), param.numel(),
                               ptr(lr_dev), ptr(step_dev), beta1, beta2, eps, float(grad_scale),
                               stream())


def step_increment(step_dev):
    lib().pld_step_increment(ptr(step_dev), stream())


def set_scalar(dev_tensor, value):
    lib().pld_set_scalar_f32(ptr(dev_tensor), float(value), stream())


class Graph:
    """A hipGraph captured from the current stream (pld_graph_*)."""

    def __init__(self):
        self.exec = None

    def capture(self, fn):
        self.begin()
        try:
            fn()
        except BaseException:
            self.end(failed=True)
            raise
        return self.end()

    def begin(self):
        """Start capturing the current stream (every launch until end() joins the graph)."""
        lib().pld_graph_begin(stream())
        _CAPTURING[0] = True
        # workspaces superseded during capture are retired from here on (the graph being built
        # may hold their pointers); the count stays only if the graph is instantiated
        _LIVE_GRAPHS[0] += 1
        return self

    def end(self, failed=False):
        _CAPTURING[0] = False
        h = C.c_void_p()
        try:
            lib().pld_graph_end(stream(), C.byref(h))
        except BaseException:
            _LIVE_GRAPHS[0] -= 1
            if failed:
                return self  # the capture's own exception is the one to report
            raise
        if failed:
            lib().pld_graph_destroy(h)
            _LIVE_GRAPHS[0] -= 1
            return self
        self.exec = h
        return self

    def launch(self):
        lib().pld_graph_launch(self.exec, stream())

    def __del__(self):
        if self.exec is not None:
            try:
                lib().pld_graph_destroy(self.exec)
            except Exception:
                pass
            self.exec = None
            try:
                _LIVE_GRAPHS[0] -= 1
                if _LIVE_GRAPHS[0] == 0:
                    _ws_retired.clear()
            except TypeError:  # interpreter shutdown: module globals already cleared
                pass


# ------------------------------------------------------------------------------------ conv
def same_pads(h, k, s):
    """TF 'same' padding: (pad_before, out)."""
    out = -(-h // s)
    total = max((out - 1) * s + k - h, 0)
    return total // 2, out


# conv product arithmetic (pld_conv_args.math): "bf16x3" (fp32 via three bf16 MFMA products,
# ~1e-5 relative per product) or "fp32" (exact fp32 MFMA). The model engines apply a policy
# (below); PLD_CONV_MATH overrides the default one.
MATH = {"fp32": 0, "bf16x3": 1}
# conv arithmetic policies: "auto" (default) = decoder bf16x3, encoder bf16x3
# where the BN after the conv normalises over >= X3_MIN_POPULATION values per channel, exact
# fp32 below (BN over a handful of pixels amplifies any rounding); "mixed" = encoder fp32,
# decoder bf16x3; "bf16x3" / "fp32" everywhere
POLICIES = ("auto", "mixed", "bf16x3", "fp32")
X3_MIN_POPULATION = 4096
CONV_MATH = [os.environ.get("PLD_CONV_MATH", "auto")]


def set_conv_math(policy):
    """Default conv policy for engines built afterwards (and for conv_args() without math=)."""
    if policy not in POLICIES:
        raise ValueError(f"conv math must be one of {POLICIES}, got {policy!r}")
    CONV_MATH[0] = policy


def conv_policy(policy=None):
    """(encoder math, decoder math) of a policy (default: the current one)."""
    policy = policy or CONV_MATH[0]
    if policy not in POLICIES:
        raise ValueError(f"conv math must be one of {POLICIES}, got {policy!r}")
    if policy == "mixed":
        return ("fp32", "bf16x3")
    if policy == "auto":
        return ("auto", "bf16x3")
    return (policy, policy)


def encoder_math(enc_math, population, threshold=None):
    """Resolve an engine's encoder math for one conv whose BN sees `population` values per
    channel (batch x output pixels); `threshold` defaults to X3_MIN_POPULATION (an engine may
    carry its own: RedWebFF.x3_min_population)."""
    if enc_math != "auto":
        return enc_math
    return "bf16x3" if population >= (threshold or X3_MIN_POPULATION) else "fp32"


def conv_args(x1, x2, kh, kw, stride, pad_t, pad_l, oh, ow, cout, in_scale=None, in_shift=None,
              in_act="none", math=None):
    n, h, w, c1 = x1.shape
    c2 = 0 if x2 is None else x2.shape[3]
    a = ConvArgs()
    a.x1 = x1.data_ptr()
    a.x2 = None if x2 is None else x2.data_ptr()
    a.c1, a.c2 = c1, c2
    a.n, a.h, a.w = n, h, w
    a.kh, a.kw, a.sh, a.sw = kh, kw, stride, stride
    a.pad_t, a.pad_l = pad_t, pad_l
    a.oh, a.ow, a.cout = oh, ow, cout
    a.in_scale = None if in_scale is None else in_scale.data_ptr()
    a.in_shift = None if in_shift is None else in_shift.data_ptr()
    a.in_act = ACT[in_act]
    a.tile = -1
    a.math = MATH[math or conv_policy()[1]]
    a._keep = (x1, x2, in_scale, in_shift)  # the struct holds raw pointers: keep owners alive
    return a


def conv_kernel_name(args, mode):
    """The main kernel a conv call with these args launches (pld_conv_kernel_name)."""
    return lib().pld_conv_kernel_name(C.byref(args), {"fwd": 0, "dgrad": 1, "wgrad": 2}[mode]) \
        .decode()


def filter_to_native(w_hwio, out=None):
    kh, kw, cin, cout = w_hwio.shape
    out = torch.empty((cout, kh, kw, cin), dtype=torch.float32, device=w_hwio.device) \
        if out is None else out
    lib().pld_filter_to_native(ptr(w_hwio), kh, kw, cin, cout, ptr(out), stream())
    return out


def filter_to_dgrad(w_hwio, out=None):
    kh, kw, cin, cout = w_hwio.shape
    out = torch.empty((cin, kh, kw, cout), dtype=torch.float32, device=w_hwio.device) \
        if out is None else out
    lib().pld_filter_to_dgrad(ptr(w_hwio), kh, kw, cin, cout, ptr(out), stream())
    return out


# ---- per-shape tile autotuning (eager only; the choice never changes results) ----
AUTOTUNE = os.environ.get("PLD_AUTOTUNE", "1") != "0"
_TILE_CACHE = {}
_CAPTURING = [False]


# The persisted schedule table of the bench workloads on MI355X (written by
# `bench.py --tune`, loaded by default by bench.py and by the parity tests of the bench's
# arithmetic): with it every conv schedule of a run is fixed before the first step, no choice
# depends on timing, and the same table governs the timed run and its gradient checks.
DEFAULT_SCHEDULES = os.path.join(os.path.dirname(os.path.abspath(__file__)), "schedules",
                                 "gfx950.json")
SCHEDULE_FORMAT = 2


def _arch():
    return torch.cuda.get_device_properties(torch.cuda.current_device()).gcnArchName \
        if torch.cuda.is_available() else "none"


def schedule_desc(math, idx):
    """Stable name of schedule `idx` (pld_conv_schedule_desc); "default" for -1 (the cost
    model's / a direct kernel's own choice)."""
    if idx < 0:
        return "default"
    d = lib().pld_conv_schedule_desc(math, idx)
    return None if d is None else d.decode()


def _schedule_index(math, desc):
    if desc == "default":
        return -1
    for i in range(lib().pld_conv_num_schedules(math)):
        if lib().pld_conv_schedule_desc(math, i).decode() == desc:
            return i
    return None


def load_tile_cache(path, arch=None):
    """Merge a schedule table written by save_tile_cache. Entries are keyed by conv shape and
    name their schedule by pld_conv_schedule_desc, so a table stays valid across library
    builds; entries whose schedule this build no longer has are dropped. Returns the number of
    entries taken (0 when the table was tuned on another GPU arch)."""
    import json
    with open(path) as f:
        d = json.load(f)
    if not isinstance(d, dict) or d.get("format") != SCHEDULE_FORMAT:
        return 0
    if d.get("arch") != (arch or _arch()):
        return 0
    taken = 0
    for k, desc in d.get("entries", []):
        k = tuple(k)
        idx = _schedule_index(k[-1], desc)
        if idx is not None:
            _TILE_CACHE[k] = idx
            taken += 1
    return taken


def save_tile_cache(path):
    import json
    entries = sorted([list(k), schedule_desc(k[-1], v)] for k, v in _TILE_CACHE.items())
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path, "w") as f:
        json.dump({"format": SCHEDULE_FORMAT, "arch": _arch(),
                   "key": ["mode", "n", "h", "w", "c1", "c2", "kh", "kw", "sh", "sw", "pad_t",
                           "pad_l", "oh", "ow", "cout", "in_prologue", "math"],
                   "entries": entries}, f, indent=0)


def use_schedule_table(path=None):
    """Fix every conv schedule from a persisted table (default: DEFAULT_SCHEDULES) and turn
    timing-based tuning off: shapes the table does not hold run the cost model's choice.
    Returns (entries taken, sha1 of the file)."""
    import hashlib
    global AUTOTUNE
    path = path or DEFAULT_SCHEDULES
    with open(path, "rb") as f:
        sha = hashlib.sha1(f.read()).hexdigest()
    _TILE_CACHE.clear()
    n = load_tile_cache(path)
    AUTOTUNE = False
    return n, sha


def _shape_key(mode, a):
    return (mode, a.n, a.h, a.w, a.c1, a.c2, a.kh, a.kw, a.sh, a.sw, a.pad_t, a.pad_l, a.oh,
            a.ow, a.cout, bool(a.in_scale), a.math)


def _skinny(a):
    return (a.cout == 1 and a.kh == 3 and a.kw == 3 and a.sh == 1 and a.c2 == 0
            and not a.in_scale and a.c1 % 4 == 0 and a.c1 <= 64)


def _patch_ok(mode, a):
    """Shapes the bf16x3 patch kernels take (pld__x3_patch_ok for the FWD view of fwd / dgrad;
    pld__x3_patch_wgrad_ok for wgrad)."""
    if a.kh != 3 or a.kw != 3 or a.sh != 1 or a.sw != 1 or a.in_scale:
        return False
    if mode == "wgrad":
        return a.c1 % 16 == 0 and a.c2 % 16 == 0 and a.cout % 4 == 0
    # fwd / dgrad (FWD view: dgrad's input is dY): one 32-channel source for all three patch
    # schedules, channels in 16s per source for the multi-chunk one
    return (a.c1 % 16 == 0 and a.c2 % 16 == 0) if mode == "fwd" else a.cout % 16 == 0


def _halo_ok(mode, a):
    """Shapes the bf16x3 row-band halo kernel takes (pld__x3_halo_ok, FWD view of fwd / dgrad):
    3x3 stride 1 'same', maps up to 56 pixels wide, channels in 8s."""
    if (a.kh != 3 or a.kw != 3 or a.sh != 1 or a.sw != 1 or a.in_scale or mode == "wgrad"
            or a.oh != a.h or a.ow != a.w or a.w > 56):
        return False
    return (a.c1 % 8 == 0 and a.c2 % 8 == 0) if mode == "fwd" else a.cout % 8 == 0


def _schedules(mode, math, a=None):
    """Schedule indices worth timing (pld_conv_args.tile): fwd/dgrad every tile x split-K
    schedule (+ the patch kernel where it applies, + the tile streams); wgrad sizes its own
    split, so only the tiles (and tile streams). Under bf16x3 the exact-fp32 schedules follow
    the bf16x3 ones. A call with an input prologue cannot stream (it would run the default)."""
    n = lib().pld_conv_num_schedules(math)
    out, patch_seen = [], False
    for i in range(n):
        c = lib().pld_conv_schedule_class(math, i)
        if c == 2 and mode == "wgrad":  # one wgrad patch schedule (it sizes its own split)
            if patch_seen:
                continue
            patch_seen = True
        if mode == "wgrad" and c not in (0, 2, 3, 5):
            continue
        if c == 5 and a is not None and a.in_scale:
            continue
        if c == 2 and (a is None or not _patch_ok(mode, a)):
            continue
        if c == 6 and (a is None or not _halo_ok(mode, a)
                       or ("halo28" in schedule_desc(math, i) and a.w > 28)):
            continue
        out.append(i)
    return out


TUNE_PASSES = max(1, int(os.environ.get("PLD_TUNE_PASSES", "2")))


def _tune(mode, a, run):
    """run(tile) launches the conv into scratch outputs; returns the fastest schedule index
    (tile x split-K for fwd/dgrad; wgrad sizes its own split, so only the tile is searched)."""
    key = _shape_key(mode, a)
    if key in _TILE_CACHE:
        return _TILE_CACHE[key]
    if not AUTOTUNE or _CAPTURING[0] or _skinny(a):
        return -1
    if lib().pld_conv_kernel_kind(C.byref(a), {"fwd": 0, "dgrad": 1, "wgrad": 2}[mode]) == 2:
        _TILE_CACHE[key] = -1  # direct VALU kernels (thin 1x1): no schedule to choose
        return -1
    st = torch.cuda.current_stream()
    scheds = _schedules(mode, a.math, a)
    # time in isolation: work queued on the engine's side streams (weight gradients, overlapped
    # branches) must not share the GPU with the candidates
    torch.cuda.synchronize()
    for t in scheds:
        run(t)  # warm-up (also sizes the workspace)
    # two timed passes over all candidates, best of the two per candidate: one noisy sample
    # (clock ramp, a neighbour's traffic) no longer decides the tile for the whole run
    times = {t: float("inf") for t in scheds}
    for _ in range(TUNE_PASSES):
        for t in scheds:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            run(t)
            run(t)
            e1.record(st)
            e1.synchronize()
            times[t] = min(times[t], e0.elapsed_time(e1))
    best = min(scheds, key=lambda t: times[t]) if scheds else -1
    _TILE_CACHE[key] = best
    return best


def _splitk_ws(args, fn):
    need = fn(C.byref(args))
    if need:
        ws = workspace(need, "splitk")
        args.ws, args.ws_bytes = ws.data_ptr(), ws.numel()
    else:
        args.ws, args.ws_bytes = None, 0


def filter_refresh(w_hwio, w_nat, w_nat_split=None, w_dg=None, w_dg_split=None):
    """pld_filter_refresh: native (+ split) and dgrad (+ split) filter copies of an HWIO weight in
    two passes; the split copies are attached to their fp32 tensors (as filter_split does)."""
    kh, kw, cin, cout = w_hwio.shape
    lib().pld_filter_refresh(ptr(w_hwio), kh, kw, cin, cout, ptr(w_nat), ptr(w_nat_split),
                             ptr(w_dg), ptr(w_dg_split), stream())
    if w_nat_split is not None:
        w_nat._pld_split = w_nat_split
    if w_dg_split is not None:
        w_dg._pld_split = w_dg_split


class _RefreshDesc(C.Structure):
    """Mirror of ``pld_filter_refresh_desc``."""
    _fields_ = [("w", C.c_void_p), ("w_nat", C.c_void_p), ("w_nat_split", C.c_void_p),
                ("w_dgrad", C.c_void_p), ("w_dgrad_split", C.c_void_p),
                ("taps", C.c_int), ("cin", C.c_int), ("cout", C.c_int),
                ("blk0", C.c_int), ("nblk", C.c_int), ("reserved", C.c_int)]


class FilterRefreshBatch:
    """Every listed filter's pld_filter_refresh in one launch (pld_filter_refresh_multi) from a
    device descriptor table built once; filters the batched path does not take (layout or
    alignment) keep their own pld_filter_refresh call. Entries: (w_hwio, w_nat, w_nat_split,
    w_dg, w_dg_split), the buffers fixed for the batch's lifetime."""

    def __init__(self, entries, device):
        self.entries = list(entries)
        descs, self.single, blk = [], [], 0
        for e in self.entries:
            w, wn, wns, wd, wds = e
            kh, kw, cin, cout = w.shape
            nb = lib().pld_filter_refresh_plan(kh, kw, cin, cout, ptr(w), ptr(wn), ptr(wns),
                                               ptr(wd), ptr(wds))
            if nb <= 0:
                self.single.append(e)
                continue
            a = [None if t is None else ptr(t).value for t in e]
            descs.append(_RefreshDesc(*a, kh * kw, cin, cout, blk, nb, 0))
            blk += nb
        self.count, self.blocks = len(descs), blk
        self.table = None
        if descs:
            arr = (_RefreshDesc * len(descs))(*descs)
            host = torch.from_numpy(np.frombuffer(bytes(arr), dtype=np.uint8).copy())
            self.table = host.to(device)
            torch.cuda.synchronize(device)
        for w, wn, wns, wd, wds in self.entries:  # the split copies ride on their fp32 tensors
            if wns is not None:
                wn._pld_split = wns
            if wds is not None:
                wd._pld_split = wds

    def __call__(self):
        if self.count:
            lib().pld_filter_refresh_multi(ptr(self.table), self.count, self.blocks, stream())
        for e in self.single:
            filter_refresh(*e)


def filter_split(w, out=None):
    """Split a [rows][K] fp32 filter (K % 8 == 0) for the bf16x3 kernel and attach the copy to
    the fp32 tensor object (w._pld_split): conv2d_fwd / conv2d_dgrad given that same tensor use
    it. The owner (engine_common._Conv.refresh) rewrites both together."""
    out = torch.empty_like(w) if out is None else out
    K_ = w.shape[-1] if w.dim() == 2 else int(np.prod(w.shape[1:]))
    rows = w.shape[0]
    lib().pld_filter_split(ptr(w), rows, K_, ptr(out), stream())
    w._pld_split = out
    return out


def _set_split(args, w):
    s = getattr(w, "_pld_split", None) if args.math == MATH["bf16x3"] else None
    args.w_split = None if s is None else s.data_ptr()


def _begin(args):
    """The caller's schedule request (-1 = tune per shape). One args object may serve the fwd,
    dgrad and wgrad of a conv: the schedule each call resolves is recorded in args._used_tile and
    args.tile is restored afterwards (_end), so a wgrad-tuned tile never leaks into the dgrad."""
    return args.tile


def _end(args, tile_in):
    args._used_tile = args.tile
    args.tile = tile_in


def _fwd_schedule(args, w_native, bias, y):
    """Resolve args.tile for a forward conv (autotuned per shape when -1) and size its split-K
    workspace."""
    if args.tile < 0:
        scratch = None

        def run(t):
            nonlocal scratch
            scratch = torch.empty_like(y) if scratch is None else scratch
            args.tile = t
            _splitk_ws(args, lib().pld_conv2d_fwd_workspace_size)
            lib().pld_conv2d_fwd(C.byref(args), ptr(w_native), ptr(bias), ptr(scratch), 0,
                                 stream())
        args.tile = _tune("fwd", args, run)
    _splitk_ws(args, lib().pld_conv2d_fwd_workspace_size)


def conv2d_fwd(args, w_native, bias, y, accumulate=False):
    tile_in = _begin(args)
    _set_split(args, w_native)
    _fwd_schedule(args, w_native, bias, y)
    lib().pld_conv2d_fwd(C.byref(args), ptr(w_native), ptr(bias), ptr(y), int(accumulate),
                         stream())
    _end(args, tile_in)
    return y


def conv2d_fwd_bn_stats(args, w_native, bias, y, mean, invstd, moving_mean=None,
                        moving_var=None, eps=1e-3, momentum=0.99):
    """conv2d_fwd + bn_stats of its output (pld_conv2d_fwd_bn_stats: the statistics gathered by
    the conv kernel's epilogue where it supports it)."""
    tile_in = _begin(args)
    _set_split(args, w_native)
    _fwd_schedule(args, w_native, bias, y)
    need = lib().pld_conv2d_fwd_bn_stats_workspace_size(C.byref(args))
    ws = workspace(need, "bnstats")
    lib().pld_conv2d_fwd_bn_stats(C.byref(args), ptr(w_native), ptr(bias), ptr(y), eps,
                                  momentum, ptr(mean), ptr(invstd), ptr(moving_mean),
                                  ptr(moving_var), ptr(ws), need, stream())
    _end(args, tile_in)
    return y


def conv2d_dgrad(args, dy, w_dgrad, dx1, dx2=None, acc1=False, acc2=False):
    tile_in = _begin(args)
    _set_split(args, w_dgrad)
    if args.tile < 0:
        s1 = s2 = None

        def run(t):
            nonlocal s1, s2
            s1 = torch.empty_like(dx1) if s1 is None else s1
            s2 = (torch.empty_like(dx2) if dx2 is not None else None) if s2 is None else s2
            args.tile = t
            _splitk_ws(args, lib().pld_conv2d_dgrad_workspace_size)
            lib().pld_conv2d_dgrad(C.byref(args), ptr(dy), ptr(w_dgrad), ptr(s1), 0, ptr(s2), 0,
                                   stream())
        args.tile = _tune("dgrad", args, run)
    _splitk_ws(args, lib().pld_conv2d_dgrad_workspace_size)
    lib().pld_conv2d_dgrad(C.byref(args), ptr(dy), ptr(w_dgrad), ptr(dx1), int(acc1), ptr(dx2),
                           int(acc2), stream())
    _end(args, tile_in)


def conv2d_wgrad(args, dy, dw, accumulate=False):
    tile_in = _begin(args)
    if args.tile < 0:
        sdw = None

        def run(t):
            nonlocal sdw
            sdw = torch.empty_like(dw) if sdw is None else sdw
            args.tile = t
            need = lib().pld_conv2d_wgrad_workspace_size(C.byref(args))
            ws = workspace(need, "wgrad") if need else None
            lib().pld_conv2d_wgrad(C.byref(args), ptr(dy), ptr(sdw), 0, ptr(ws), need, stream())
        args.tile = _tune("wgrad", args, run)
    need = lib().pld_conv2d_wgrad_workspace_size(C.byref(args))
    ws = workspace(need, "wgrad") if need else None
    lib().pld_conv2d_wgrad(C.byref(args), ptr(dy), ptr(dw), int(accumulate), ptr(ws), need,
                           stream())
    _end(args, tile_in)


def channel_sum(x, rows, c, out, accumulate=False, ws_key="reduce"):
    """out[c] (+)= sum over rows of x[rows, c]; ws_key: the workspace to use (a call on another
    stream than the BN reductions needs its own)."""
    ws = workspace(lib().pld_channel_reduce_workspace_size(rows, c), ws_key)
    lib().pld_channel_sum(ptr(x), rows, c, ptr(out), int(accumulate), ptr(ws), stream())


# -------------------------------------------------------------------------------------- BN
def bn_stats(x, rows, c, mean, invstd, moving_mean=None, moving_var=None, eps=1e-3,
             momentum=0.99):
    ws = workspace(lib().pld_channel_reduce_workspace_size(rows, c), "reduce")
    lib().pld_bn_stats(ptr(x), rows, c, eps, momentum, ptr(mean), ptr(invstd), ptr(moving_mean),
                       ptr(moving_var), ptr(ws), stream())


def bn_apply(x, rows, c, mean, invstd, gamma, beta, act, y, gate=None, hw=0):
    lib().pld_bn_apply(ptr(x), rows, c, ptr(mean), ptr(invstd), ptr(gamma), ptr(beta), ACT[act],
                       ptr(gate), hw, ptr(y), stream())


def bn_bwd(x, dy, rows, c, mean, invstd, gamma, beta, act, dx, dgamma, dbeta, gate=None,
           addn=None, hw=0, dx_accumulate=False, param_accumulate=False):
    ws = workspace(lib().pld_channel_reduce_workspace_size(rows, c), "reduce")
    lib().pld_bn_bwd(ptr(x), ptr(dy), rows, c, ptr(mean), ptr(invstd), ptr(gamma), ptr(beta),
                     ACT[act], ptr(gate), ptr(addn), hw, ptr(dx), int(dx_accumulate),
                     ptr(dgamma), ptr(dbeta), int(param_accumulate), ptr(ws), stream())


def bn_bwd_coeffs(x, dy, rows, c, mean, invstd, gamma, beta, act, dgamma, dbeta, k12,
                  param_accumulate=False):
    """pld_bn_bwd's reductions + finalize: dgamma, dbeta and k12 [2c] for pgemm_bn_bwd."""
    ws = workspace(lib().pld_channel_reduce_workspace_size(rows, c), "reduce")
    lib().pld_bn_bwd_coeffs(ptr(x), ptr(dy), rows, c, ptr(mean), ptr(invstd), ptr(gamma),
                            ptr(beta), ACT[act], ptr(dgamma), ptr(dbeta), int(param_accumulate),
                            ptr(k12), ptr(ws), stream())


def pgemm_ok(k, n):
    return bool(lib().pld_pgemm_ok(int(k), int(n)))


def pgemm_pays(k, n):
    """Where the fused pgemm beats the unfused pair (tools/pgemm_micro.py, MI355X, 448^2 batch
    32): filter K x N <= 4096 floats, i.e. it stays in the scalar cache that feeds the FMAs
    (1a/2a/2b project, 2a/2b/3a expand dgrad: 26-176 us saved each); at 144 x 40 and 240 x 40
    the filter streams from L2 per 16-wide chunk and the bf16x3 MFMA pair is faster."""
    return pgemm_ok(k, n) and k * n <= 4096


def pgemm_bn_act(x, rows, k, mean, invstd, gamma, beta, act, w, n, y, gate=None, hw=0,
                 accumulate=False):
    """y [rows, n] = (act(bn(x)) * gate[img]) . w^T  (w [n][k])."""
    lib().pld_pgemm_bn_act(ptr(x), rows, k, ptr(mean), ptr(invstd), ptr(gamma), ptr(beta),
                           ACT[act], ptr(gate), hw, ptr(w), n, ptr(y), int(accumulate), stream())


def pgemm_bn_bwd(x, dy, rows, k, mean, invstd, gamma, beta, act, k12, w, n, y,
                 accumulate=False):
    """y [rows, n] = bn_bwd(x, dy; k12) . w^T  (w [n][k])."""
    lib().pld_pgemm_bn_bwd(ptr(x), ptr(dy), rows, k, ptr(mean), ptr(invstd), ptr(gamma),
                           ptr(beta), ACT[act], ptr(k12), ptr(w), n, ptr(y), int(accumulate),
                           stream())


def bn_add_apply(x, rows, c, mean, invstd, gamma, beta, res, act, y):
    lib().pld_bn_add_apply(ptr(x), rows, c, ptr(mean), ptr(invstd), ptr(gamma), ptr(beta),
                           ptr(res), ACT[act], ptr(y), stream())


def bn_scale_add_apply(x, rows, c, mean, invstd, gamma, beta, sample_scale, hw, res, act, y):
    """y = act(bn(x) * sample_scale[row // hw] + res) (pld_bn_scale_add_apply; sample_scale None:
    bn_add_apply)."""
    lib().pld_bn_scale_add_apply(ptr(x), rows, c, ptr(mean), ptr(invstd), ptr(gamma), ptr(beta),
                                 ptr(sample_scale), hw, ptr(res), ACT[act], ptr(y), stream())


def bn_bwd_scaled(x, dy, rows, c, mean, invstd, gamma, beta, act, sample_scale, hw, dx, dgamma,
                  dbeta, dx_accumulate=False, param_accumulate=False):
    """bn_bwd of dy * sample_scale[row // hw] (pld_bn_bwd_scaled)."""
    ws = workspace(lib().pld_channel_reduce_workspace_size(rows, c), "reduce")
    lib().pld_bn_bwd_scaled(ptr(x), ptr(dy), rows, c, ptr(mean), ptr(invstd), ptr(gamma),
                            ptr(beta), ACT[act], ptr(sample_scale), hw, ptr(dx),
                            int(dx_accumulate), ptr(dgamma), ptr(dbeta), int(param_accumulate),
                            ptr(ws), stream())


def bn_add_bwd(x, dy, rows, c, mean, invstd, gamma, beta, res, act, dx, dres, dgamma, dbeta,
               dx_accumulate=False, dres_accumulate=False, param_accumulate=False):
    ws = workspace(lib().pld_channel_reduce_workspace_size(rows, c), "reduce")
    lib().pld_bn_add_bwd(ptr(x), ptr(dy), rows, c, ptr(mean), ptr(invstd), ptr(gamma),
                         ptr(beta), ptr(res), ACT[act], ptr(dx), int(dx_accumulate), ptr(dres),
                         int(dres_accumulate), ptr(dgamma), ptr(dbeta), int(param_accumulate),
                         ptr(ws), stream())


def maxpool2d_fwd(x, k, s, pad_t, pad_l, y, argmax=None):
    n, h, w, c = x.shape
    oh, ow = y.shape[1], y.shape[2]
    lib().pld_maxpool2d_fwd(ptr(x), n, h, w, c, k, s, pad_t, pad_l, oh, ow, ptr(y), ptr(argmax),
                            stream())
    return y


def maxpool2d_bwd(dy, argmax, k, s, pad_t, pad_l, dx, accumulate=False):
    n, h, w, c = dx.shape
    oh, ow = dy.shape[1], dy.shape[2]
    lib().pld_maxpool2d_bwd(ptr(dy), ptr(argmax), n, h, w, c, k, s, pad_t, pad_l, oh, ow, ptr(dx),
                            int(accumulate), stream())
    return dx


def channel_affine_act(x, rows, c, scale, shift, act, y):
    lib().pld_channel_affine_act(ptr(x), rows, c, ptr(scale), ptr(shift), ACT[act], ptr(y),
                                 stream())


# ------------------------------------------------------------------------------ resampling
def upsample2x_fwd(x, y, bn=None, act="none"):
    """bn = (mean, invstd, gamma, beta): x is the pre-BN tensor; BN + act is applied to each
    tap as it is read (the activation before the upsampling is never materialised)."""
    n, h, w, c = x.shape
    if bn is None:
        lib().pld_upsample2x_fwd(ptr(x), n, h, w, c, ptr(y), stream())
    else:
        mean, invstd, gamma, beta = bn
        lib().pld_upsample2x_fwd_bn(ptr(x), n, h, w, c, ptr(mean), ptr(invstd), ptr(gamma),
                                    ptr(beta), ACT[act], ptr(y), stream())
    return y


def upsample2x_bwd(dy, dx, accumulate=False):
    n, h, w, c = dx.shape
    lib().pld_upsample2x_bwd(ptr(dy), n, h, w, c, ptr(dx), int(accumulate), stream())
    return dx


def upconv_fwd(x, bn, wt, bias, y):
    """y [n,2h,2w,1] = conv3x3(up2x(relu(bn(x)))) + bias; bn = (mean, invstd, gamma, beta)."""
    n, h, w, c = x.shape
    mean, invstd, gamma, beta = bn
    lib().pld_upconv_fwd(ptr(x), n, h, w, c, ptr(mean), ptr(invstd), ptr(gamma), ptr(beta),
                         ptr(wt), ptr(bias), ptr(y), stream())
    return y


def upconv_wgrad(x, bn, dy, dw):
    n, h, w, c = x.shape
    mean, invstd, gamma, beta = bn
    need = lib().pld_upconv_wgrad_workspace_size(c)
    ws = workspace(need, "upconv")
    lib().pld_upconv_wgrad(ptr(x), n, h, w, c, ptr(mean), ptr(invstd), ptr(gamma), ptr(beta),
                           ptr(dy), ptr(dw), ptr(ws), need, stream())


def upconv_bwd(x, bn, wt, dy, dact, dw=None, dx=None, dgamma=None, dbeta=None,
               dx_accumulate=False, param_accumulate=False):
    """The fused last stage's backward in one pass over (x, dy): dact [n,h,w,c] (gradient of
    relu(bn(x))), dw [3,3,c,1] if given, and if dx is given the BN + ReLU backward of x
    (dx, dgamma, dbeta) with its channel reductions taken in the same pass."""
    n, h, w, c = x.shape
    mean, invstd, gamma, beta = bn
    need = lib().pld_upconv_bwd_workspace_size(c)
    ws = workspace(need, "upconv")
    lib().pld_upconv_bwd(ptr(x), n, h, w, c, ptr(mean), ptr(invstd), ptr(gamma), ptr(beta),
                         ptr(wt), ptr(dy), ptr(dact), ptr(dw), ptr(dx), int(dx_accumulate),
                         ptr(dgamma), ptr(dbeta), int(param_accumulate), ptr(ws), need,
                         stream())


def upconv_dgrad(dy, wt, dact):
    """dact [n,h,w,c] = up2x^T(conv3x3^T(dy)) for dy [n,2h,2w,1], wt [3,3,c,1] (HWIO)."""
    n, h, w, c = dact.shape
    lib().pld_upconv_dgrad(ptr(dy), n, h, w, c, ptr(wt), ptr(dact), stream())


def residual_add(a, sample_scale, b, y):
    n = a.shape[0]
    lib().pld_residual_add(ptr(a), ptr(sample_scale), ptr(b), n, a.numel() // n, ptr(y),
                           stream())


def dropconnect_scales(scales, rate, seed, step, layer, image_offset=0):
    """step: an int, or a device int64 tensor (graph-replayable counter)."""
    if isinstance(step, torch.Tensor):
        lib().pld_dropconnect_scales_dev(ptr(scales), scales.numel(), float(rate), seed,
                                         ptr(step), layer, image_offset, stream())
    else:
        lib().pld_dropconnect_scales(ptr(scales), scales.numel(), float(rate), seed, step, layer,
                                     image_offset, stream())


def dropconnect_scales_multi(scales, rates, layers, seed, step, image_offset=0):
    """scales [len(layers), n]: row s = dropconnect_scales(n, rates[s], ..., layers[s]) in one
    launch; step: an int or a device int64 tensor."""
    import ctypes
    nl = len(layers)
    assert scales.dim() == 2 and scales.shape[0] == nl and scales.is_contiguous()
    assert len(rates) == nl
    dev = isinstance(step, torch.Tensor)
    # one launch per DC_MAX_LAYERS rows (the kernel's parameter block; EfficientNetB0 has 16)
    for s0 in range(0, nl, DC_MAX_LAYERS):
        m = min(DC_MAX_LAYERS, nl - s0)
        r = (ctypes.c_float * m)(*[float(x) for x in rates[s0:s0 + m]])
        l = (ctypes.c_int * m)(*[int(x) for x in layers[s0:s0 + m]])
        lib().pld_dropconnect_scales_multi(ptr(scales[s0:s0 + m]), scales.shape[1], m,
                                           ctypes.cast(r, ctypes.c_void_p),
                                           ctypes.cast(l, ctypes.c_void_p), seed,
                                           0 if dev else step, ptr(step) if dev else None,
                                           image_offset, stream())


DC_MAX_LAYERS = 32  # pld_dropconnect_scales_multi rows per launch (resample.hip)


def bn_train_coeffs(mean, invstd, gamma, beta, scale, shift):
    """Training-mode BN as act-free affine coefficients (scale = gamma*invstd, shift = beta -
    mean*scale): the consuming conv's input prologue (conv_args in_scale / in_shift)."""
    lib().pld_bn_train_coeffs(ptr(mean), ptr(invstd), ptr(gamma), ptr(beta), gamma.numel(),
                              ptr(scale), ptr(shift), stream())


def channel_pad_affine(x, cout, y, scale=None, shift=None):
    """y [.., cout] = [x*scale + shift | 0] of x [.., cin] (the stem's widened input)."""
    cin = x.shape[-1]
    lib().pld_channel_pad_affine(ptr(x), x.numel() // cin, cin, cout, ptr(scale), ptr(shift),
                                 ptr(y), stream())
    return y


def bn_inference_coeffs(gamma, beta, mmean, mvar, scale, shift, eps=1e-3):
    lib().pld_bn_inference_coeffs(ptr(gamma), ptr(beta), ptr(mmean), ptr(mvar), gamma.numel(),
                                  eps, ptr(scale), ptr(shift), stream())


def scale_per_sample(x, sample_scale, y, accumulate=False):
    n = x.shape[0]
    lib().pld_scale_per_sample(ptr(x), ptr(sample_scale), n, x.numel() // n, ptr(y),
                               int(accumulate), stream())


# ------------------------------------------------------------------------- depthwise / SE
def dwconv_fwd(x, wdw, k, s, pad_t, pad_l, y, bn=None, act="none"):
    """bn = (mean, invstd, gamma, beta): x is the producer's pre-BN tensor and the training-mode
    BN + act is applied as the pixels are read (no materialised activation)."""
    n, h, w, c = x.shape
    _, oh, ow, _ = y.shape
    if bn is None:
        lib().pld_dwconv_fwd(ptr(x), n, h, w, c, ptr(wdw), k, s, pad_t, pad_l, oh, ow, ptr(y),
                             stream())
    else:
        mean, invstd, gamma, beta = bn
        lib().pld_dwconv_fwd_bn(ptr(x), n, h, w, c, ptr(wdw), k, s, pad_t, pad_l, oh, ow,
                                ptr(mean), ptr(invstd), ptr(gamma), ptr(beta), ACT[act], ptr(y),
                                stream())


def dwconv_fwd_bn_stats(x, wdw, k, s, pad_t, pad_l, y, ybn, bn=None, act="none", eps=1e-3,
                        momentum=0.99):
    """dwconv_fwd + the batch statistics of y for the BN after it: ybn = (mean, invstd,
    moving_mean, moving_var) written like bn_stats (gathered in the tiled kernel's epilogue)."""
    n, h, w, c = x.shape
    _, oh, ow, _ = y.shape
    need = lib().pld_dwconv_fwd_bn_stats_workspace_size(n, oh, ow, c, s)
    ws = workspace(need, "bnstats")
    mean, invstd, gamma, beta = bn if bn is not None else (None,) * 4
    ym, yi, ymm, ymv = ybn
    lib().pld_dwconv_fwd_bn_stats(ptr(x), n, h, w, c, ptr(wdw), k, s, pad_t, pad_l, oh, ow,
                                  ptr(mean), ptr(invstd), ptr(gamma), ptr(beta), ACT[act],
                                  ptr(y), eps, momentum, ptr(ym), ptr(yi), ptr(ymm), ptr(ymv),
                                  ptr(ws), need, stream())


def dwconv_dgrad(dy, wdw, k, s, pad_t, pad_l, dx, accumulate=False):
    n, h, w, c = dx.shape
    _, oh, ow, _ = dy.shape
    lib().pld_dwconv_dgrad(ptr(dy), n, h, w, c, ptr(wdw), k, s, pad_t, pad_l, oh, ow, ptr(dx),
                           int(accumulate), stream())


def dwconv_dgrad_bn_bwd(dy, wdw, k, s, pad_t, pad_l, dact, x, bn, act, dgamma, dbeta, k12,
                        dx=None, accumulate=False, dx_accumulate=False, param_accumulate=False):
    """dwconv_dgrad into dact with the backward of the BN + act that produced the depthwise input
    (x: that BN's input; bn = (mean, invstd, gamma, beta)) fused: its reductions in the dgrad's
    epilogue, then dgamma/dbeta/k12, and dx (the BN input gradient) when given."""
    n, h, w, c = dact.shape
    _, oh, ow, _ = dy.shape
    need = lib().pld_dwconv_dgrad_bn_bwd_workspace_size(n, h, w, c, s)
    ws = workspace(need, "dwbnb")
    mean, invstd, gamma, beta = bn
    lib().pld_dwconv_dgrad_bn_bwd(ptr(dy), n, h, w, c, ptr(wdw), k, s, pad_t, pad_l, oh, ow,
                                  ptr(dact), int(accumulate), ptr(x), ptr(mean), ptr(invstd),
                                  ptr(gamma), ptr(beta), ACT[act], ptr(dx), int(dx_accumulate),
                                  ptr(dgamma), ptr(dbeta), int(param_accumulate), ptr(k12),
                                  ptr(ws), need, stream())


def se_fwd(a, w1, b1, w2, b2, pooled, z1, gate, bn=None, act="swish"):
    """bn = (mean, invstd, gamma, beta): `a` is the pre-BN tensor; the squeeze applies BN + act."""
    n, h, w, c = a.shape
    cse = w1.shape[-1]
    ws = workspace(lib().pld_se_workspace_size(n, h * w, c, cse), "se")
    if bn is None:
        lib().pld_se_fwd(ptr(a), n, h * w, c, cse, ptr(w1), ptr(b1), ptr(w2), ptr(b2),
                         ptr(pooled), ptr(z1), ptr(gate), ptr(ws), stream())
    else:
        mu, inv, g, b = bn
        lib().pld_se_fwd_bn(ptr(a), ptr(mu), ptr(inv), ptr(g), ptr(b), ACT[act], n, h * w, c,
                            cse, ptr(w1), ptr(b1), ptr(w2), ptr(b2), ptr(pooled), ptr(z1),
                            ptr(gate), ptr(ws), stream())


def se_bwd(dy, a, w1, w2, z1, gate, addn, bn=None, act="swish"):
    n, h, w, c = a.shape
    cse = w1.shape[-1]
    ws = workspace(lib().pld_se_workspace_size(n, h * w, c, cse), "se")
    if bn is None:
        lib().pld_se_bwd(ptr(dy), ptr(a), n, h * w, c, cse, ptr(w1), ptr(w2), ptr(z1),
                         ptr(gate), ptr(addn), ptr(ws), stream())
    else:
        mu, inv, g, b = bn
        lib().pld_se_bwd_bn(ptr(dy), ptr(a), ptr(mu), ptr(inv), ptr(g), ptr(b), ACT[act], n,
                            h * w, c, cse, ptr(w1), ptr(w2), ptr(z1), ptr(gate), ptr(addn),
                            ptr(ws), stream())


def se_bwd_bn_full(dy, x, bn, w1, w2, z1, gate, addn, dx, dgamma, dbeta, act="swish",
                   dx_accumulate=False, param_accumulate=False):
    """SE backward (addn) + the block BN's backward (dx, dgamma, dbeta) with the BN reductions
    gathered by the SE squeeze sweep over (x, dy): pld_se_bwd_bn_full."""
    n, h, w, c = x.shape
    cse = w1.shape[-1]
    need = lib().pld_se_bwd_bn_full_workspace_size(n, h * w, c, cse)
    ws = workspace(need, "se_bn")
    mu, inv, g, b = bn
    lib().pld_se_bwd_bn_full(ptr(dy), ptr(x), ptr(mu), ptr(inv), ptr(g), ptr(b), ACT[act], n,
                             h * w, c, cse, ptr(w1), ptr(w2), ptr(z1), ptr(gate), ptr(addn),
                             ptr(dx), int(dx_accumulate), ptr(dgamma), ptr(dbeta),
                             int(param_accumulate), ptr(ws), need, stream())


# -------------------------------------------------------------------------------- sampler
def sampler_candidates(R, strategy):
    return lib().pld_sampler_candidates(R, SAMPLER[strategy])


def sampler_compact(mask, gt, valid_idx, nvalid, gt_minmax):
    B, H, W = mask.shape
    ws = workspace(lib().pld_sampler_compact_workspace_size(B, H, W), "compact")
    lib().pld_sampler_compact(ptr(mask), B, H, W, ptr(gt), ptr(valid_idx), ptr(nvalid),
                              ptr(gt_minmax), ptr(ws), stream())


def sampler_draw(nvalid, n_cand, L, seed, step, image_offset, draws):
    """step: an int, or a device int64 tensor (graph-replayable counter)."""
    B = nvalid.shape[0]
    if isinstance(step, torch.Tensor):
        lib().pld_sampler_draw_dev(ptr(nvalid), B, n_cand, L, seed, ptr(step), image_offset,
                                   ptr(draws), stream())
    else:
        lib().pld_sampler_draw(ptr(nvalid), B, n_cand, L, seed, step, image_offset, ptr(draws),
                               stream())


def sampler_rank(gt, valid_idx, nvalid, gt_minmax, draws, R, L, strategy, out):
    B, H, W = gt.shape
    sid = SAMPLER[strategy]
    ws = workspace(lib().pld_sampler_workspace_size(B, H, W, R, L, sid), "sampler")
    lib().pld_sampler_rank(ptr(gt), ptr(valid_idx), ptr(nvalid), ptr(gt_minmax), ptr(draws), B,
                           H, W, R, L, sid, ptr(out), ptr(ws), stream())
    return out


# ---- test-pass metrics (pld_ordinal_error / pld_dcg_ratio) ----
def ordinal_error(pred, gt, idx0, idx1):
    """pred, gt: [n, hw] float32 device tensors; idx0/idx1: int32 device indices -> [n] float64."""
    n, hw = pred.shape[0], pred[0].numel()
    assert gt.shape[0] == n and gt[0].numel() == hw and idx0.numel() == idx1.numel()
    assert idx0.dtype == torch.int32 and idx1.dtype == torch.int32
    out = torch.empty(n, dtype=torch.float64, device=pred.device)
    lib().pld_ordinal_error(ptr(_f32(pred)), ptr(_f32(gt)), n, hw, ptr(idx0), ptr(idx1),
                            idx0.numel(), ptr(out), stream())
    return out


def dcg_ratio(pred, gt, ids):
    """pred, gt: [n, hw] float32 device tensors; ids: int32 device list -> [n] float64."""
    n, hw = pred.shape[0], pred[0].numel()
    assert gt.shape[0] == n and gt[0].numel() == hw and ids.dtype == torch.int32
    out = torch.empty(n, dtype=torch.float64, device=pred.device)
    lib().pld_dcg_ratio(ptr(_f32(pred)), ptr(_f32(gt)), n, hw, ptr(ids), ids.numel(), ptr(out),
                        stream())
    return out


# ---- HR-WSI resizing (pld_resize_bilinear / pld_resize_nearest) ----
def resize(x, oh, ow, method="bilinear", out=None):
    """x: [n, h, w, c] float32 device tensor -> [n, oh, ow, c] (tf.image.resize, TF2 semantics)."""
    n, h, w, c = x.shape
    out = torch.empty((n, oh, ow, c), dtype=torch.float32, device=x.device) if out is None else out
    fn = lib().pld_resize_bilinear if method == "bilinear" else lib().pld_resize_nearest
    fn(ptr(_f32(x.contiguous())), n, h, w, c, oh, ow, ptr(out), stream())
    return out
