"""Root-cause tool for the hipGraph replay drift.

Records the C-ABI calls of one eager ReplicaTrainer step (every pld_* status call with its
exact ctypes arguments, on the trainer's stream), then replays that call list in several
forms against an eagerly stepped twin and reports the first step whose state differs:

  eager      the recorded calls re-issued eagerly (sanity: must match)
  single     every call captured into its own hipGraph, the graphs launched in order
  whole      all calls captured into one hipGraph (what ReplicaTrainer.capture() does)
  bisect     find the shortest contiguous run of calls [s, m) which, captured as ONE graph
             (every other call in its own graph), still drifts

Run it with DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 (the runtime default) and =0 to compare.
Writes gpurun_out/graph_bisect_<pc>.json."""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from pldepth_amd import _lib  # noqa: E402
from pldepth_amd.trainer import ReplicaTrainer  # noqa: E402

MODEL = os.environ.get("GB_MODEL", "ff_effnet")
B, H, L, R = 2, 64, 5, 20
STEPS = int(os.environ.get("GB_STEPS", "6"))
torch.cuda.set_device(0)
rng = np.random.default_rng(0)
X = torch.from_numpy(rng.random((B, H, H, 3)).astype(np.float32)).cuda()
GT = torch.from_numpy(rng.random((B, H, H)).astype(np.float32)).cuda()
MASK = torch.from_numpy((rng.random((B, H, H)) < 0.9).astype(np.float32)).cuda()
LIB = _lib.lib()
GRAPH_FNS = {"pld_graph_begin", "pld_graph_end", "pld_graph_launch", "pld_graph_destroy"}


def make():
    t = ReplicaTrainer((H, H, 3), B, L, R, 1, seed=0, model=MODEL)
    t.set_batch(X, GT, MASK)
    return t


def state(t):
    e = t.engine
    d = {"step": t.step_dev.float(), "y": t.y_true, "loss": t.loss, "params": e.params.buf,
         "m": t.m, "v": t.v, "vhat": t.vhat, "stats": e.stats.buf, "grads": e.grads.buf}
    for c in e.convs:
        if c.trainable:
            for k in ("w_nat", "w_dg", "w_nat_x3", "w_dg_x3"):
                if getattr(c, k) is not None:
                    d[f"{c.name}.{k}"] = getattr(c, k)
    for k, v in e.act.items():
        d["act." + k] = v
    return {k: v.detach().clone() for k, v in d.items()}


def differs(sa, sb):
    return [k for k in sa if not torch.allclose(sa[k], sb[k], rtol=1e-4, atol=1e-6)]


def record(t):
    """One eager step of t with every C-ABI status call recorded as (name, fn, args)."""
    calls, saved = [], {}
    for name in list(vars(LIB)):
        fn = getattr(LIB, name)
        if not name.startswith("pld_") or name in GRAPH_FNS or name in _lib._NON_STATUS:
            continue
        saved[name] = fn

        def rec(*args, _n=name, _f=fn):
            # byref(ConvArgs) objects keep their struct alive; copy structs so later edits of
            # the engine's args objects cannot change the recorded call
            args = tuple(_clone(a) for a in args)
            calls.append((_n, _f, args))
            return _f(*args)
        setattr(LIB, name, rec)
    try:
        t.step_eager(0.01)
        t.synchronize()
    finally:
        for name, fn in saved.items():
            setattr(LIB, name, fn)
    return calls


def _clone(a):
    if type(a).__name__ == "CArgObject":  # byref(struct)
        s = a._obj
        c = type(s)()
        C.pointer(c)[0] = s
        return C.byref(c)
    return a


def issue(calls):
    for _, fn, args in calls:
        fn(*args)


def capture(t, calls):
    g = C.c_void_p()
    st = C.c_void_p(t.stream.cuda_stream)
    LIB.pld_graph_begin(st)
    try:
        issue(calls)
    finally:
        LIB.pld_graph_end(st, C.byref(g))
    return g


def run(parts):
    """parts: list of (lo, hi, as_graph). Returns (first drifting step or None, keys)."""
    a, b = make(), make()
    a.step_eager(0.01)
    b.step_eager(0.01)
    a.synchronize()
    b.synchronize()
    calls = record(a)
    b.step_eager(0.01)
    b.synchronize()
    st = C.c_void_p(a.stream.cuda_stream)
    plan = []
    with torch.cuda.stream(a.stream):
        for lo, hi, as_graph in parts:
            plan.append(("g", capture(a, calls[lo:hi])) if as_graph else ("e", calls[lo:hi]))
    torch.cuda.synchronize()
    result = (None, [])
    for i in range(STEPS):
        with torch.cuda.stream(a.stream):
            for kind, obj in plan:
                if kind == "g":
                    LIB.pld_graph_launch(obj, st)
                else:
                    issue(obj)
        a.synchronize()
        b.step_eager(0.01)
        b.synchronize()
        bad = differs(state(a), state(b))
        if bad:
            result = (i, bad[:12])
            break
    for kind, obj in plan:
        if kind == "g":
            LIB.pld_graph_destroy(obj)
    del a, b
    torch.cuda.empty_cache()
    return result, calls


def main():
    pc = os.environ.get("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "<unset>")
    out = {"packet_capture_env": pc, "model": MODEL}
    (r, calls) = run([(0, 10 ** 9, False)])
    n = len(calls)
    out["n_calls"] = n
    out["calls"] = [c[0] for c in calls]
    out["eager"] = r
    print("calls", n, "eager:", r, flush=True)
    single = [(i, i + 1, True) for i in range(n)]
    out["single"] = run(single)[0]
    print("single:", out["single"], flush=True)
    out["whole"] = run([(0, n, True)])[0]
    print("whole:", out["whole"], flush=True)
    if out["single"][0] is not None:
        # one-call graphs drift too: find the calls whose graph replay differs from their eager
        # launch (every other call eager)
        def drifts1(lo, hi):
            parts = [(0, lo, False)] + [(i, i + 1, True) for i in range(lo, hi)] + \
                    [(hi, n, False)]
            return run(parts)[0][0] is not None
        lo_m, hi_m = 1, n  # smallest m with one-call graphs over [0, m) drifting
        while lo_m < hi_m:
            mid = (lo_m + hi_m) // 2
            if drifts1(0, mid):
                hi_m = mid
            else:
                lo_m = mid + 1
        m = lo_m
        lo_s, hi_s = 0, m - 1  # largest s with [s, m) drifting
        while lo_s < hi_s:
            mid = (lo_s + hi_s + 1) // 2
            if drifts1(mid, m):
                lo_s = mid
            else:
                hi_s = mid - 1
        s = lo_s
        out["single_window"] = [s, m, [c[0] for c in calls[s:m]]]
        print("graph-replayed calls that drift", s, m, [c[0] for c in calls[s:m]], flush=True)
        if m - s == 1:  # the call's arguments, for the report
            out["single_window_args"] = [repr(a) for a in calls[s][2]]
            a0 = calls[s][2][0]
            if type(a0).__name__ == "CArgObject":
                st = a0._obj
                out["single_window_struct"] = {f: repr(getattr(st, f)) for f, _ in st._fields_}
    if out["whole"][0] is not None and out["single"][0] is None:
        def drifts(lo, hi):
            parts = [(i, i + 1, True) for i in range(lo)] + [(lo, hi, True)] + \
                    [(i, i + 1, True) for i in range(hi, n)]
            return run(parts)[0][0] is not None
        lo_m, hi_m = 1, n  # smallest m with [0, m) drifting
        while lo_m < hi_m:
            mid = (lo_m + hi_m) // 2
            if drifts(0, mid):
                hi_m = mid
            else:
                lo_m = mid + 1
        m = lo_m
        lo_s, hi_s = 0, m - 1  # largest s with [s, m) drifting
        while lo_s < hi_s:
            mid = (lo_s + hi_s + 1) // 2
            if drifts(mid, m):
                lo_s = mid
            else:
                hi_s = mid - 1
        s = lo_s
        out["window"] = [s, m, [c[0] for c in calls[s:m]]]
        print("minimal drifting window", s, m, [c[0] for c in calls[s:m]], flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    with open(f"gpurun_out/graph_bisect_{MODEL}_pc{pc}.json", "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
