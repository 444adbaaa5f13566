"""PLDepth training-step throughput on MI355X (BASELINE.json metric: images/s at 448x448,
ranking_size=5, ff_effnet, per-GPU batch 32, Info sampler, Adam-AMSGrad; synthetic data).

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (one rank per GPU)

A step = GPU ranking sampler + ff_effnet forward + ListMLE + backward + (RCCL all-reduce) +
Adam-AMSGrad + filter refresh, on a resident synthetic batch, replayed from hipGraphs. Rank 0
prints one JSON line. See DESIGN.md §Measurement for the roofline and cpu_baseline definitions.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32 dense peak (spec)
BF16_MFMA_PEAK_TFLOPS = 2500.0  # dense bf16 MFMA peak (spec, no sparsity)
# per conv kernel family (pld_conv_kernel_kind): peak in fp32-equivalent algorithmic TFLOP/s;
# bf16x3 spends three bf16 MFMA products per fp32 product.
KIND_PEAK = {0: FP32_MFMA_PEAK_TFLOPS, 1: BF16_MFMA_PEAK_TFLOPS / 3.0, 2: FP32_MFMA_PEAK_TFLOPS}
KIND_NAME = {0: "fp32_mfma", 1: "bf16x3_mfma", 2: "direct_valu"}


def log(msg):
    """progress on stderr (stdout carries only rank 0's JSON line)"""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def synthetic_batch(B, H, W, seed):
    """x ~ U[0,1); gt = smooth 8-bit-quantised depth field; mask ~ Bernoulli(0.9)."""
    rng = np.random.default_rng(seed)
    x = rng.random((B, H, W, 3), dtype=np.float32)
    yy, xx = np.meshgrid(np.linspace(0, 1, H), np.linspace(0, 1, W), indexing="ij")
    gt = np.empty((B, H, W), np.float32)
    for b in range(B):
        f = np.zeros((H, W))
        for _ in range(6):
            fy, fx = rng.uniform(0.3, 3.0, 2)
            ph = rng.uniform(0, 2 * np.pi, 2)
            f += rng.uniform(0.2, 1.0) * np.sin(2 * np.pi * fy * yy + ph[0]) * \
                np.cos(2 * np.pi * fx * xx + ph[1])
        f = (f - f.min()) / (f.max() - f.min())
        gt[b] = np.round(255 * f).astype(np.float32) / np.float32(255)
    mask = (rng.random((B, H, W)) < 0.9).astype(np.float32)
    return x, gt, mask


def profile_conv(trainer, lr, replays=None):
    """One eager step with HIP events around every conv call (on the stream the kernels run on).
    Returns one record per call: (kernel name, family kind, mode, algorithmic FLOPs, algorithmic
    HBM bytes, seconds). The kernel name is the main kernel the call launched
    (pld_conv_kernel_name: the name rocprof lists); a call's time includes the split-K slab
    reduction it may add. `replays` (a list) collects (kernel name, closure re-issuing the call
    with the same arguments) per conv call, for replay_dominant."""
    import ctypes
    from pldepth_amd import kernels as K
    from pldepth_amd._lib import lib
    st = trainer.stream
    recs = []
    # conv2d_fwd_bn_stats: the conv + its output's BN statistics (gathered in the thin kernel's
    # epilogue, else a stats pass): the call's time includes the statistics
    orig = {n: getattr(K, n) for n in ("conv2d_fwd", "conv2d_dgrad", "conv2d_wgrad",
                                       "conv2d_fwd_bn_stats")}
    mode_of = {"conv2d_fwd": 0, "conv2d_dgrad": 1, "conv2d_wgrad": 2, "conv2d_fwd_bn_stats": 0}

    def flops_of(a):
        # fwd, dX and dW of one conv are the same contraction: 2 * outputs * taps * Cin * Cout
        return 2.0 * a.n * a.oh * a.ow * a.cout * a.kh * a.kw * (a.c1 + a.c2)

    def bytes_of(a):
        # the two activations the contraction reads / writes (input x | dX, output y | dY) and
        # the filter (w | dW), each once: 4 B per element
        return 4.0 * (a.n * a.h * a.w * (a.c1 + a.c2) + a.n * a.oh * a.ow * a.cout
                      + a.kh * a.kw * (a.c1 + a.c2) * a.cout)

    def wrap(name):
        fn = orig[name]

        def w(args, *rest, **kw):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            r = fn(args, *rest, **kw)
            e1.record(st)
            saved = args.tile  # classify by the schedule the call actually ran
            args.tile = getattr(args, "_used_tile", saved)
            kind = lib().pld_conv_kernel_kind(ctypes.byref(args), mode_of[name])
            kname = lib().pld_conv_kernel_name(ctypes.byref(args), mode_of[name]).decode()
            args.tile = saved
            recs.append((kname, kind, mode_of[name], flops_of(args), bytes_of(args), e0, e1))
            if replays is not None:  # the same call again, for the graph-replayed timing
                replays.append((kname, flops_of(args), bytes_of(args),
                                lambda: fn(args, *rest, **kw)))
            return r
        return w

    # the fused BN+ReLU -> upsample -> final 3x3 conv (csrc/upconv.hip): direct VALU kernels.
    # Algorithmic FLOPs are the conv's own (2 per MAC over the 2x map, per fwd / dX / dW pass:
    # the SURVEY §8d count); bytes: x (or dact) + the 1-channel 2x map + the filter.
    up_orig = {n: getattr(K, n) for n in ("upconv_fwd", "upconv_wgrad", "upconv_dgrad",
                                          "upconv_bwd")}

    def up_wrap(name, mode):
        fn = up_orig[name]

        def w(*args, **kw):
            # dgrad: (dy, wt, dact) -> dact is [n,h,w,c]; bwd: (x, bn, wt, dy, dact, ...)
            x = args[2] if name == "upconv_dgrad" else args[0]
            n_, h_, w_, c_ = x.shape
            passes = 2 if name == "upconv_bwd" else 1  # bwd: dX and dW in one pass
            fl = passes * 2.0 * n_ * (2 * h_) * (2 * w_) * 9 * c_
            by = 4.0 * (n_ * h_ * w_ * c_ * (2 if name == "upconv_bwd" else 1)
                        + n_ * 4 * h_ * w_ + 9 * c_)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            r = fn(*args, **kw)
            e1.record(st)
            recs.append((name + "_kernel", 2, mode, fl, by, e0, e1))
            return r
        return w

    for n in orig:
        setattr(K, n, wrap(n))
    for n, m in (("upconv_fwd", 0), ("upconv_dgrad", 1), ("upconv_wgrad", 2),
                 ("upconv_bwd", 1)):
        setattr(K, n, up_wrap(n, m))
    # one stream: each kernel's events bracket it alone (the engine's decoder weight gradients
    # otherwise overlap the rest of the backward on a side stream)
    overlap = getattr(trainer.engine, "overlap_wgrad", False)
    trainer.engine.overlap_wgrad = False
    try:
        trainer.step_eager(lr)
        st.synchronize()
    finally:
        trainer.engine.overlap_wgrad = overlap
        for n, f in orig.items():
            setattr(K, n, f)
        for n, f in up_orig.items():
            setattr(K, n, f)
    return [(n, k, m, f, b, e0.elapsed_time(e1) / 1e3) for n, k, m, f, b, e0, e1 in recs]


# kernels.py wrapper -> op family (the step-level byte floor and the PMC traffic per family)
def _family(fn):
    if fn.startswith(("conv2d", "pgemm", "upconv", "channel_sum", "filter_split")):
        return "conv"
    if fn.startswith(("bn_", "channel_affine")):
        return "batchnorm"
    if fn.startswith("dwconv"):
        return "depthwise"
    if fn.startswith("se_"):
        return "squeeze_excite"
    if fn.startswith(("upsample", "maxpool", "residual", "scale_per_sample", "dropconnect")):
        return "resample_residual"
    if fn.startswith(("sampler", "listmle")):
        return "sampler_listmle"
    return "optimizer_refresh"  # adam, filter_refresh, step / scalar updates


def step_byte_floor(trainer, lr):
    """Step-level algorithmic byte floor: one eager step with every kernels.py entry point
    wrapped; each call counts every distinct tensor it is handed ONCE (its inputs read once, its
    outputs written once; a tensor it reads and writes in place counts once; library scratch
    workspaces not at all). Summed per op family = "each activation written once and read once
    per consumer" for the launch sequence this build runs. Returns {family: bytes}, total."""
    from pldepth_amd import kernels as K
    ws_ptrs = lambda: {b.data_ptr() for b in K._ws_cache.values()}
    depth, seen, fam = [0], [None], {}
    orig_ptr = K.ptr

    def ptr(t):
        if t is not None and depth[0] > 0 and seen[0] is not None:
            seen[0][t.data_ptr()] = t.numel() * t.element_size()
        return orig_ptr(t)

    names = [n for n, f in vars(K).items() if callable(f) and not n.startswith("_")
             and getattr(f, "__module__", None) == K.__name__ and n not in (
                 "ptr", "stream", "workspace", "conv_args", "conv_policy", "encoder_math",
                 "set_conv_math", "same_pads", "sampler_candidates", "pgemm_ok", "pgemm_pays",
                 "load_tile_cache", "save_tile_cache", "Graph", "schedule_desc",
                 "use_schedule_table")]
    saved = {n: getattr(K, n) for n in names}

    def wrap(n, f):
        def w(*args, **kw):
            outer = depth[0] == 0
            if outer:
                seen[0] = {}
            depth[0] += 1
            try:
                for a in list(args) + list(kw.values()):
                    keep = getattr(a, "_keep", None)  # ConvArgs: x1, x2, in_scale, in_shift
                    if keep is not None:
                        for t in keep:
                            if t is not None:
                                seen[0][t.data_ptr()] = t.numel() * t.element_size()
                return f(*args, **kw)
            finally:
                depth[0] -= 1
                if outer:
                    skip = ws_ptrs()
                    fam[_family(n)] = fam.get(_family(n), 0) + sum(
                        v for p, v in seen[0].items() if p not in skip)
                    seen[0] = None
        return w

    K.ptr = ptr
    for n in names:
        setattr(K, n, wrap(n, saved[n]))
    try:
        trainer.step_eager(lr)
        trainer.synchronize()
    finally:
        K.ptr = orig_ptr
        for n, f in saved.items():
            setattr(K, n, f)
    return fam, sum(fam.values())


def attach_step_traffic(roof, path, workload):
    """The measured side of the byte floor: per-family HBM bytes of one eager step from the
    committed PMC profile (tools/pmc_step_family.py), only when its workload matches."""
    if path and not os.path.isabs(path):
        path = os.path.join(os.path.dirname(os.path.abspath(__file__)), path)
    try:
        with open(path) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return
    if t.get("workload") != workload:
        return
    alg = roof["step_bytes_algorithmic"]
    roof["step_bytes_measured"] = {
        "total": t["total_bytes"], "by_family": t["by_family"], "profile": path,
        "over_algorithmic": round(t["total_bytes"] / alg["total"], 3),
        "note": "PMC FETCH_SIZE x2 (gfx950 64-B tally) + WRITE_SIZE of one eager step; FETCH "
                "counts Infinity-Cache hits too, so these are upper bounds on HBM bytes"}


def attach_traffic(roof, path, workload):
    """roofline.traffic = HBM bytes per launch of the dominant kernel from the committed PMC
    profile (tools/dominant_traffic.py), only when that profile measured the same kernel on the
    same workload; otherwise it stays null."""
    if path and not os.path.isabs(path):  # relative to the repository, whatever the cwd
        path = os.path.join(os.path.dirname(os.path.abspath(__file__)), path)
    try:
        with open(path) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return
    if t.get("kernel") != roof["kernel"] or (workload and t.get("workload") != workload):
        roof["traffic_note"] = "profile does not match this run's dominant kernel / workload"
        return
    roof["traffic"] = t["hbm_bytes_per_launch"]
    roof["traffic_algorithmic"] = t["algorithmic_bytes_per_launch"]
    roof["traffic_over_algorithmic"] = t["hbm_over_algorithmic"]
    if "mfma_busy" in t:  # SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)
        roof["mfma_busy"] = t["mfma_busy"]


HBM_PEAK_TBS = 8.0  # MI355X_MICROARCH.md: HBM3E peak (spec)


def _graph_ms(trainer, calls, reps):
    """Capture `calls` (in order) into one hipGraph on the trainer's stream, replay it once to
    warm, then `reps` times between HIP events on that stream: ms per replay."""
    from pldepth_amd import kernels as K
    st = trainer.stream
    with torch.cuda.stream(st):
        g = K.Graph().capture(lambda: [c() for c in calls])
        g.launch()
        st.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(reps):
            g.launch()
        e1.record(st)
        e1.synchronize()
    del g
    return e0.elapsed_time(e1) / reps


def replay_dominant(trainer, replays, roof, reps=5):
    """The dominant kernel's launches of one step (every conv call whose main kernel it is, same
    arguments and schedules, in step order) captured into one hipGraph on the trainer's stream
    and replayed `reps` times between HIP events on that stream: its duration without host launch
    gaps (roofline.graph_replay). The launches are also split by the bound their own shape sets
    (roofline.by_bound): a launch whose algorithmic FLOP per byte lies below the ridge point
    peak / 8 TB/s is HBM-bound and is scored in TB/s against the HBM peak, the rest against the
    MFMA peak; each group is captured and timed on its own.
    The replays re-issue the step's own convs after the timed region: their outputs are
    rewritten by the next step, and the BN moving statistics that the statistics-gathering calls
    update are saved before and restored after, so no later use sees replay state."""
    calls = [(f, b, c) for n, f, b, c in replays if n == roof["kernel"]]
    if not calls:
        return
    eng = trainer.engine
    saved = eng.stats.buf.clone() if getattr(eng, "stats", None) is not None else None
    try:
        ms = _graph_ms(trainer, [c for _, _, c in calls], reps)
        ridge = roof["peak"] * 1e12 / (HBM_PEAK_TBS * 1e12)  # FLOP per byte
        groups = {"mfma": [x for x in calls if x[0] / x[1] >= ridge],
                  "hbm": [x for x in calls if x[0] / x[1] < ridge]}
        by_bound = {}
        for bound, grp in groups.items():
            if not grp:
                continue
            gms = _graph_ms(trainer, [c for _, _, c in grp], reps)
            fl, by = sum(x[0] for x in grp), sum(x[1] for x in grp)
            e = {"launches": len(grp), "ms_per_step": round(gms, 4),
                 "flops_per_step": fl, "bytes_per_step": by}
            if bound == "mfma":
                ach = fl / (gms * 1e-3) / 1e12
                e.update(achieved=round(ach, 3), peak=roof["peak"], unit="TFLOP/s",
                         frac=round(ach / roof["peak"], 4))
            else:
                ach = by / (gms * 1e-3) / 1e12
                e.update(achieved=round(ach, 3), peak=HBM_PEAK_TBS, unit="TB/s",
                         frac=round(ach / HBM_PEAK_TBS, 4),
                         note="algorithmic bytes (each operand once + the output) / time")
            by_bound[bound] = e
    finally:
        if saved is not None:
            eng.stats.buf.copy_(saved)
            torch.cuda.synchronize()
    d = roof["dominant"]
    ach = d["flops_per_step"] / (ms * 1e-3) / 1e12
    roof["graph_replay"] = {
        "achieved": round(ach, 3), "frac": round(ach / roof["peak"], 4),
        "ms_per_step": round(ms, 4), "avg_us": round(ms * 1e3 / len(calls), 2),
        "timing": (f"the {len(calls)} launches of {roof['kernel']} of one step captured into one "
                   f"hipGraph, {reps} replays between HIP events on the trainer's stream")}
    roof["by_bound"] = by_bound
    roof["by_bound_rule"] = (f"per launch: algorithmic FLOP/B >= ridge {ridge:.1f} "
                             f"(= {roof['peak']} TFLOP/s / {HBM_PEAK_TBS} TB/s) -> mfma, else hbm")
    # live headline (until a matching in-step rocprof profile replaces it: attach_graph_frac)
    roof["achieved"], roof["frac"] = round(ach, 3), round(ach / roof["peak"], 4)
    roof["headline"] = "graph_replay (live)"


def attach_graph_frac(roof, path, workload):
    """The dominant kernel's fraction of peak as rocprof measured it inside the timed whole-step
    graph replays (the decoder weight gradients then overlap the encoder backward on a side
    stream, so its launches share the GPU), from the kernel-trace summary committed at the same
    HEAD and workload: roofline.rocprof_step_replay."""
    if path and not os.path.isabs(path):
        path = os.path.join(os.path.dirname(os.path.abspath(__file__)), path)
    try:
        with open(path) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return
    d = roof.get("dominant", {})
    if t.get("kernel") != roof["kernel"] or t.get("workload") != workload or \
            t.get("launches_per_step") != d.get("launches_per_step"):
        return
    ach = d["flops_per_step"] / (t["ms_per_step"] * 1e-3) / 1e12
    roof["rocprof_step_replay"] = {"ms_per_step": t["ms_per_step"], "achieved": round(ach, 3),
                                   "frac": round(ach / roof["peak"], 4), "source": t["source"]}
    # the in-step figure (the timed steps' own execution, where the decoder
    # weight gradients share the GPU on a side stream) is the headline; the live graph replay of
    # the kernel's launches alone stays under graph_replay
    roof["achieved"], roof["frac"] = roof["rocprof_step_replay"]["achieved"], \
        roof["rocprof_step_replay"]["frac"]
    roof["headline"] = "rocprof_step_replay (in-step, committed kernel trace at this workload)"


def conv_roofline(recs, traffic_profile=None):
    """roofline object. Top level = the DOMINANT kernel (the conv kernel name with the largest
    summed time in the profiled step): achieved = its algorithmic FLOPs / its measured time (the
    eager HIP-event time here, kept under `eager`; replay_dominant replaces the headline with the
    graph-replayed time, attach_graph_frac with the in-step rocprof time when a kernel trace of
    this workload is committed), peak = the MFMA peak of its arithmetic. `family` keeps the whole conv family (FLOP-weighted blend
    of the families' peaks: the same FLOPs with every launch at its own family's peak). traffic
    (PMC HBM bytes) cannot be read inside this process: null here; the PMC pass of the same
    command is committed under profiles/ (traffic_profile) with the algorithmic bytes beside it."""
    fam, by_name = {}, {}
    for name, kind, mode, fl, by, sec in recs:
        d = fam.setdefault(kind, [0.0, 0.0, 0])
        d[0] += fl
        d[1] += sec
        d[2] += 1
        e = by_name.setdefault(name, {"kind": kind, "flops": 0.0, "bytes": 0.0, "sec": 0.0,
                                      "launches": 0, "modes": set()})
        e["flops"] += fl
        e["bytes"] += by
        e["sec"] += sec
        e["launches"] += 1
        e["modes"].add(("fwd", "dgrad", "wgrad")[mode])
    fl = sum(v[0] for v in fam.values())
    sec = sum(v[1] for v in fam.values())
    t_peak = sum(v[0] / (KIND_PEAK[k] * 1e12) for k, v in fam.items())
    dname = max(by_name, key=lambda n: by_name[n]["sec"])
    d = by_name[dname]
    d_ach = d["flops"] / d["sec"] / 1e12
    d_peak = KIND_PEAK[d["kind"]]
    dominant = {
        "kernel": dname, "family": KIND_NAME[d["kind"]], "modes": sorted(d["modes"]),
        "launches_per_step": d["launches"], "flops_per_step": d["flops"],
        "bytes_per_step": d["bytes"], "avg_us": round(d["sec"] / d["launches"] * 1e6, 2),
        "ms_per_step": round(d["sec"] * 1e3, 4), "achieved_tflops": round(d_ach, 3),
        "peak_tflops": round(d_peak, 1), "frac": round(d_ach / d_peak, 4),
        "achieved_gbps": round(d["bytes"] / d["sec"] / 1e9, 1),
    }
    return {
        "bound": "mfma",
        "kernel": dname,
        "achieved": round(d_ach, 3), "peak": round(d_peak, 1), "unit": "TFLOP/s",
        "frac": round(d_ach / d_peak, 4),
        "headline": "eager (live)",
        "eager": {"achieved": round(d_ach, 3), "frac": round(d_ach / d_peak, 4),
                  "ms_per_step": dominant["ms_per_step"],
                  "note": "HIP events around each conv call of one eager step"},
        "traffic": None,
        "traffic_profile": traffic_profile,
        "dominant": dominant,
        "family": {
            "kernel": "conv family: conv_x3_kernel / conv_x3_patch* (bf16x3 MFMA) + "
                      "conv_igemm_kernel (fp32 MFMA) + direct VALU kernels (Cout=1 3x3, thin 1x1)",
            "achieved": round(fl / sec / 1e12, 3), "peak": round(fl / t_peak / 1e12, 3),
            "frac": round((fl / sec) / (fl / t_peak), 4), "launches": sum(v[2] for v in
                                                                          fam.values()),
            "flops_per_step": fl, "ms_per_step": round(sec * 1e3, 3),
            "families": {KIND_NAME[k]: {"tflop": round(v[0] / 1e12, 4),
                                        "ms": round(v[1] * 1e3, 3), "launches": v[2],
                                        "achieved": round(v[0] / v[1] / 1e12, 2),
                                        "peak": round(KIND_PEAK[k], 1)}
                         for k, v in sorted(fam.items())},
        },
        "kernels": {n: {"ms": round(v["sec"] * 1e3, 3), "launches": v["launches"],
                        "achieved_tflops": round(v["flops"] / v["sec"] / 1e12, 2)}
                    for n, v in sorted(by_name.items(), key=lambda kv: -kv[1]["sec"])},
    }


def cpu_baseline(H, W, L, R, model="ff_effnet", seconds_budget=25.0):
    """The oracle (torch-CPU fp32 restatement of the full step + numpy sampler restatement),
    8 threads as the reference's init_tensorflow(num_threads=8), on a bounded sample."""
    sys.path.insert(0, ROOT)
    from oracle import listmle as LM
    from oracle import sampler as S
    torch.set_num_threads(8)
    B = 2
    x, gt, mask = synthetic_batch(B, H, W, seed=123)
    if model == "ff_effnet":
        from oracle import effnet as OM
        w = _cpu_weights(H, W)
    else:
        from oracle import redweb as OM
        from pldepth_amd.models.redweb_ff import preprocess_input
        x = preprocess_input(x)
        rng = np.random.default_rng(0)
        w = {}
        for n, shp, _ in OM.param_specs():
            if n.endswith(("/gamma", "moving_variance")):
                w[n] = np.ones(shp, np.float32)
            elif len(shp) == 1:
                w[n] = np.zeros(shp, np.float32)
            else:
                lim = np.sqrt(6.0 / (shp[0] * shp[1] * (shp[2] + shp[3])))
                w[n] = rng.uniform(-lim, lim, shp).astype(np.float32)
    P = {k: torch.tensor(v) for k, v in w.items()}
    names = sorted(OM.trainable_names(P))
    fwd = (lambda Q, xx: OM.forward(Q, xx)) if model == "ff_effnet" else \
        (lambda Q, xx: OM.forward(Q, xx, preprocessed=True))
    from oracle.adam import adam_amsgrad_step
    adam = {k: [np.zeros(P[k].shape, np.float32) for _ in range(3)] for k in names}
    np.random.seed(0)

    def one_step(step):
        ys = [S.sample_masked_point_batch("info", mask[b], gt[b], R, L)[0] for b in range(B)]
        y = np.stack(ys)
        Q = {k: (v.clone().requires_grad_(True) if k in names else v) for k, v in P.items()}
        out = fwd(Q, torch.tensor(x))
        loss, dpred = LM.hourglass_nll(y, out.detach().numpy(), B, L)
        out.backward(torch.tensor(dpred, dtype=torch.float32))
        for k in names:  # Adam-AMSGrad (oracle/adam.py) on every trainable tensor
            p, *st = adam_amsgrad_step(P[k].numpy(), Q[k].grad.numpy(), *adam[k], lr=1e-3,
                                       step=step)
            P[k] = torch.from_numpy(p)
            adam[k] = st

    one_step(1)  # warm-up
    n_steps, t_total = 0, 0.0
    while n_steps < 10 and t_total < seconds_budget:
        t0 = time.perf_counter()
        one_step(n_steps + 2)
        t_total += time.perf_counter() - t0
        n_steps += 1
    return {"value": B * n_steps / t_total, "unit": "images/s",
            "cores": len(os.sched_getaffinity(0)), "threads": torch.get_num_threads(),
            "kind": "port",
            "sample": f"{n_steps} timed full train steps after 1 warm-up (numpy Info sampler + "
                      f"torch-CPU fp32 {model} fwd/bwd + ListMLE + Adam-AMSGrad), batch {B}, "
                      f"{H}x{W}, L={L}, R={R}, torch.set_num_threads(8)"}


def loss_parity(tr, lr, threads=16):
    """The metric's second half, "ListMLE loss delta vs TF2": one more step of the benchmark's
    own trainer (eager, same batch, the next step's sampler rankings and drop-connect masks),
    and the oracle's fp64 restatement of the reference forward (oracle/effnet.py or
    oracle/redweb.py, training-mode BN, the step's drop-connect scales injected) + ListMLE
    (oracle/listmle.py: depth_utils.py:39-61 + tfr ListMLE) on the same weights, images and
    y_true. Checker only: rank 0 at N=1, after the timed region, like cpu_baseline()."""
    sys.path.insert(0, ROOT)
    from oracle import listmle as LM
    eng = tr.engine
    weights = eng.get_weights()  # the weights this step's forward runs with
    tr.step_eager(lr)
    tr.synchronize()
    torch.cuda.synchronize()
    loss = tr.loss_value()
    pred = eng.act["pred"].double().cpu()
    x = eng.act["input"].double().cpu()
    y = tr.y_true.cpu().numpy()
    B, R, L = y.shape[0], y.shape[1], y.shape[2]
    P = {k: torch.tensor(v, dtype=torch.float64) for k, v in weights.items()}
    nthreads = torch.get_num_threads()
    torch.set_num_threads(max(1, min(threads, len(os.sched_getaffinity(0)))))
    t0 = time.perf_counter()
    try:
        with torch.no_grad():
            if eng.__class__.__name__ == "RedWebFF":
                from oracle import redweb as OR
                pred_ref = OR.forward(P, x, preprocessed=True)
            else:
                from oracle import effnet as OE
                drop = {blk["name"]: blk["drop"].double().cpu() for blk in eng.blocks
                        if blk.get("residual") and blk.get("rate", 0) > 0 and eng.drop_connect}
                pred_ref = OE.forward(P, x, drop_scales=drop or None)
    finally:
        torch.set_num_threads(nthreads)
    loss_ref, _ = LM.hourglass_nll(y, pred_ref.numpy(), B, L)
    return {
        "loss": loss, "loss_oracle_fp64": float(loss_ref),
        "loss_delta": abs(loss - loss_ref) / abs(loss_ref),
        "pred_delta": float((pred - pred_ref).abs().max() / pred_ref.abs().max()),
        "lists": B * R, "oracle_seconds": round(time.perf_counter() - t0, 1),
        "how": "one extra eager step of the bench trainer (its own batch, sampler rankings and "
               "drop-connect masks) vs the fp64 oracle forward + ListMLE on the same weights; "
               "delta = |loss - oracle| / |oracle|, pred_delta = max|dpred| / max|pred|",
    }


def _cpu_weights(H, W):
    # the engine's initialiser, run on CPU buffers (no GPU needed)
    from pldepth_amd.models import effnet_ff as E

    class _CPU(E.EffNetFF):
        def __init__(self):
            self.H, self.W, self.B = H, W, 1
            self.device = torch.device("cpu")
            self.params, self.frozen, self.stats = E.FlatStore(), E.FlatStore(), E.FlatStore()
            self.bns, self.convs = [], []
            self._build_spec()
            for s in (self.params, self.frozen, self.stats):
                s.materialize("cpu")

        def set_weights(self, w):
            for store in (self.params, self.frozen, self.stats):
                for name, shape, _ in store.specs:
                    store[name].copy_(torch.as_tensor(np.asarray(w[name], np.float32)))

    e = _CPU()
    e.init_weights(0)
    return e.get_weights()


def run_config(model, H, B, L, R, sampling_type, steps, warmup, rank, world, pg, graph=True):
    """Build a replica for one workload, warm it up (the first step is eager: it tunes conv
    schedules and sizes workspaces, then the step is captured), time `steps` graph replays
    bracketed by barrier + synchronize. Returns (trainer, seconds)."""
    from pldepth_amd.trainer import ReplicaTrainer
    tr = ReplicaTrainer((H, H, 3), B, L, R, sampling_type, seed=0, rank=rank,
                        world_size=world, process_group=pg, model=model)
    x, gt, mask = synthetic_batch(B, H, H, seed=1000 + rank)
    if model == "ff_redweb":
        x = tr.engine.preprocess(x)  # the data pipeline's caffe preprocessing (PLDepth.py:169)
    tr.set_batch(torch.from_numpy(x).cuda(), torch.from_numpy(gt).cuda(),
                 torch.from_numpy(mask).cuda())
    lr = 0.01
    log(f"{model} {H}x{H} B={B} L={L} R={R}: first (eager) step")
    tr.step_eager(lr)
    torch.cuda.synchronize()
    if graph:
        log("capture")
        tr.capture()
    for _ in range(max(warmup - 1, 0)):
        tr.step(lr)
    torch.cuda.synchronize()

    def barrier():
        if world > 1:
            import torch.distributed as dist
            dist.barrier()
        torch.cuda.synchronize()

    barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        tr.step(lr)
    tr.synchronize()
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        import torch.distributed as dist
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return tr, elapsed


# BASELINE.json configs measured beside the headline (1 GPU): (key, model, L, R)
EXTRA_CONFIGS = [
    ("cfg3_ff_resnet", "ff_redweb", 5, 100),
    ("cfg5_ff_effnet_L64_R1000", "ff_effnet", 64, 1000),
]


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n, argv):
    """`bench.py --gpus N` started without a launcher (no WORLD_SIZE in the environment): run
    the N ranks as ONE child process, `torch.distributed.run --nproc-per-node N` on 127.0.0.1
    (each rank pins LOCAL_RANK to its GPU), and return its exit code. The parent never touches
    the GPU (no HIP call before or after), it only waits; rank 0's JSON line reaches stdout
    through the child."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node", str(n), "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "4")
    return subprocess.call(cmd, env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--size", type=int, default=448)
    ap.add_argument("--ranking-size", type=int, default=5)
    ap.add_argument("--rankings-per-image", type=int, default=100)
    ap.add_argument("--sampling-type", type=int, default=1)
    ap.add_argument("--model", default="ff_effnet", choices=["ff_effnet", "ff_redweb"],
                    help="ff_redweb = the ResNet-50 backbone (BASELINE cfg3 'ff_resnet')")
    ap.add_argument("--no-graph", action="store_true",
                    help="step eagerly (no hipGraph capture): the host-launch-bound comparison")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="torch.distributed backend for N > 1 (nccl = RCCL; gloo rehearses the "
                         "path with ranks sharing one GPU)")
    ap.add_argument("--no-cpu-baseline", action="store_true",
                    help="skip the CPU legs (cpu_baseline timing and the loss-delta check)")
    ap.add_argument("--no-loss-parity", action="store_true",
                    help="skip the ListMLE loss delta vs the fp64 oracle (loss_parity)")
    ap.add_argument("--no-extra-configs", action="store_true",
                    help="skip the cfg3 (ff_resnet) and cfg5 (L=64, R=1000) lines (1 GPU only)")
    ap.add_argument("--conv-math", default="auto", choices=["auto", "mixed", "bf16x3", "fp32"],
                    help="conv arithmetic policy (kernels.conv_policy): auto = decoder bf16x3, "
                         "encoder bf16x3 where the BN sees >= 4096 values per channel (all of "
                         "them at 448x448 batch 32); mixed = encoder fp32, decoder bf16x3")
    ap.add_argument("--traffic-profile", default="profiles/r06c_pmc_dominant.json",
                    help="PMC traffic of the dominant kernel (tools/dominant_traffic.py, committed "
                         "from the same HEAD and workload): fills roofline.traffic when its kernel "
                         "and workload match this run's")
    ap.add_argument("--graph-profile", default="profiles/r06c_dominant_graph.json",
                    help="rocprof time of the dominant kernel inside the whole-step graph replays "
                         "(roofline.rocprof_step_replay)")
    ap.add_argument("--step-traffic-profile", default="profiles/r06c_pmc_step_family.json",
                    help="PMC HBM bytes of one eager step per op family "
                         "(tools/pmc_step_family.py): roofline.step_bytes_measured")
    ap.add_argument("--schedules", default="",
                    help="persisted conv schedule table (default: pldepth_amd/schedules/"
                         "gfx950.json): every conv schedule fixed before the first step, no "
                         "timing-dependent choice in the run")
    ap.add_argument("--tune", default="",
                    help="autotune the schedules by timing instead (each candidate timed alone "
                         "on a drained device) and write the table to this path")
    ap.add_argument("--dist-timeout", type=float, default=600.0,
                    help="seconds before a collective (or the rendezvous) that a rank never "
                         "joins raises and ends the job with a non-zero status")
    ap.add_argument("--debug-fail-rank", type=int, default=-1, help=argparse.SUPPRESS)
    a = ap.parse_args()

    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(a.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    from pldepth_amd.dp import exit_on_failure
    exit_on_failure(lambda: run(a, world), world)


def run(a, world):
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    assert world == a.gpus, f"--gpus {a.gpus} but WORLD_SIZE={world}"
    # one rank per GPU; ranks beyond the visible GPUs share them (the gloo rehearsal of the
    # N > 1 path on a 1-GPU box: tests/test_bench_gpu.py)
    dev = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(dev)
    pg = None
    if world > 1:
        import torch.distributed as dist
        from pldepth_amd import dp
        # bounded: a rank that dies or never arrives ends the job (non-zero) within the timeout
        # instead of leaving the others blocked in a collective
        pg = dp.init_group(a.backend, rank, world, device=torch.device("cuda", dev),
                           timeout_s=a.dist_timeout)
    # what the process group actually holds (the SCALE record shows RCCL saw N ranks)
    ranks_seen = dist.get_world_size() if world > 1 else 1
    backend_seen = str(dist.get_backend()) if world > 1 else None
    if a.debug_fail_rank >= 0 and rank == a.debug_fail_rank:
        log(f"--debug-fail-rank: rank {rank} exits before the first step")
        os._exit(3)

    from pldepth_amd.build import LIB  # noqa: F401  (the built library must be present)
    from pldepth_amd import kernels as K
    K.set_conv_math(a.conv_math)
    sched = {"mode": "tuned in this run"}
    path = a.schedules or K.DEFAULT_SCHEDULES
    if not a.tune and os.path.exists(path):
        n_sched, sha = K.use_schedule_table(path)
        sched = {"mode": "table", "table": os.path.relpath(path, ROOT), "sha1": sha,
                 "entries": n_sched}
        if n_sched == 0:  # tuned on another arch / format: nothing taken
            sched["mode"] = "default (table not applicable: 0 entries taken; cost-model schedules)"

    H = a.size
    B, L, R = a.batch, a.ranking_size, a.rankings_per_image
    tr, elapsed = run_config(a.model, H, B, L, R, a.sampling_type, a.steps, a.warmup, rank,
                             world, pg, graph=not a.no_graph)
    loss = tr.loss_value()
    value = world * B * a.steps / elapsed
    dist_check = None
    if world > 1:
        # every replica applied the same all-reduced gradients: parameters equal bit for bit
        from pldepth_amd import dp
        same, sums = dp.replicas_identical(tr.engine.params.buf, pg)
        dist_check = {"replicas_identical": same, "param_checksums": sums,
                      "rccl_version": dp.rccl_version() if a.backend == "nccl" else None,
                      "timeout_s": a.dist_timeout,
                      # decoder buckets all-reduced while the encoder backward runs
                      # (trainer dp_overlap; PLD_DP_OVERLAP=0: after the backward)
                      "dp_overlap": tr.dp_overlap}

    # dominant conv kernel + conv family: algorithmic FLOPs / measured duration (HIP events on
    # the trainer's stream, one eager step)
    log(f"timed: {1e3 * elapsed / a.steps:.3f} ms/step; profiling")
    replays = []
    recs = profile_conv(tr, 0.01, replays)
    flops_img = tr.engine.conv_flops_per_image()
    roof = conv_roofline(recs, a.traffic_profile)
    replay_dominant(tr, replays, roof)
    del replays
    workload = (f"{a.model} train step {H}x{H}, per-GPU batch {B}, ranking_size {L}, "
                f"rankings_per_image {R}, sampler {tr.strategy}, Adam-AMSGrad")
    attach_traffic(roof, a.traffic_profile, workload)
    roof["step_frac"] = round(value / world * flops_img / 1e12 / roof["family"]["peak"], 4)
    fam, total = step_byte_floor(tr, 0.01)
    roof["step_bytes_algorithmic"] = {
        "total": total, "by_family": dict(sorted(fam.items(), key=lambda kv: -kv[1])),
        "definition": "per launch, every distinct tensor the call is handed counted once (inputs "
                      "read once, outputs written once), summed over one step's launches"}
    attach_step_traffic(roof, a.step_traffic_profile, workload)
    attach_graph_frac(roof, a.graph_profile, workload)
    out = {
        "metric": "images/sec (448x448, ranking_size=5) at 1/2/4/8 GPU; ListMLE loss delta vs TF2",
        "value": round(value, 3),
        "unit": "images/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(1e3 * elapsed / a.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp32 (bf16x3 MFMA)",
        "data": "synthetic (U[0,1) RGB, smooth 8-bit depth, Bernoulli(0.9) mask; Keras-default "
                "random-init weights)",
        "config": {"workload": workload,
                   "model": a.model, "global_batch": world * B, "input": f"{H}x{H}",
                   "ranking_size": L, "rankings_per_image": R,
                   "parallelism": f"dp{world}", "graph": not a.no_graph,
                   "backend": backend_seen, "ranks_seen": ranks_seen,
                   "gpus_visible": torch.cuda.device_count()},
        "conv_math": {"policy": a.conv_math, "encoder": tr.engine.enc_math,
                      "decoder": tr.engine.dec_math},
        "roofline": roof,
        "loss": loss,
        "distributed": dist_check,
        "schedules": sched,
    }
    if rank == 0 and world == 1 and not a.no_cpu_baseline and not a.no_loss_parity:
        log("loss parity vs the fp64 oracle")
        par = loss_parity(tr, 0.01)
        out["loss_delta"] = par["loss_delta"]
        out["loss_parity"] = par
    del tr
    if world == 1 and not a.no_extra_configs and a.model == "ff_effnet" and H == 448:
        extra = {}
        for key, model, el, er in EXTRA_CONFIGS:
            t2, el_s = run_config(model, H, B, el, er, a.sampling_type, a.steps, a.warmup,
                                  rank, world, pg, graph=not a.no_graph)
            extra[key] = {"value": round(B * a.steps / el_s, 3), "unit": "images/s",
                          "ms_per_step": round(1e3 * el_s / a.steps, 3), "model": model,
                          "input": f"{H}x{H}", "batch": B, "ranking_size": el,
                          "rankings_per_image": er, "sampler": t2.strategy,
                          "loss": t2.loss_value()}
            del t2
            torch.cuda.empty_cache()
        out["extra_configs"] = extra
    if a.tune and rank == 0:
        K.save_tile_cache(a.tune)
        out["schedules"]["written"] = a.tune
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        log("cpu baseline")
        out["cpu_baseline"] = cpu_baseline(H, H, L, R, a.model)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
