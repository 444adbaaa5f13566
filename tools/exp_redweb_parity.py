"""Experiment: which ff_redweb convs put gradient tensors over the strict
1e-3 bar at the bench's batch 32 (448x448, 'auto' policy, the bench's schedule table), and what
running them exact fp32 costs.

For each variant (RedWebFF.exact_fwd_extra / exact_bwd name prefixes): one HIP forward + ListMLE
+ backward, the HIP ReLU branches read after the forward, the fp64 oracle gradient along THOSE
branches (flip-aware, as tests/test_configs_gpu.py::test_batch32_bench_policy), and the per-tensor
errors next to the fp32 restatement's (along its own branches, computed once). Also the eager
fwd+bwd time. Writes gpurun_out/redweb_parity.json.

    python tools/exp_redweb_parity.py [variant ...]
"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import listmle as LM  # noqa: E402
from oracle import redweb as OR  # noqa: E402
from pldepth_amd import kernels as K  # noqa: E402
from pldepth_amd.models.redweb_ff import RedWebFF, preprocess_input  # noqa: E402

TOL = 1e-3
FFL_DOWN = ("ffl0/block_down", "ffl1/block_down", "ffl2/block_down")
VARIANTS = {
    "auto": ((), ()),
    "conv5_fwd": (("conv5",), ()),
    "conv5_fwdbwd": (("conv5",), ("conv5",)),
    "ffl_down_fwd": (FFL_DOWN, ()),
    "ffl_down_fwdbwd": (FFL_DOWN, FFL_DOWN),
    "ffl_fwdbwd": (("ffl",), ("ffl",)),
    "conv5+ffl_down_fwdbwd": (("conv5",) + FFL_DOWN, ("conv5",) + FFL_DOWN),
    "dec_all_fwdbwd": (("ffl", "aol"), ("ffl", "aol")),
    # the HIP backward fed the fp64 forward's dL/dpred (the fp32 restatement's input) instead of
    # its own: separates the backward's arithmetic from the forward's error carried by dpred
    "auto_dref": ((), ()),
    # every conv of the step exact fp32 (the HIP exact-fp32 kernels): what an fp32 HIP path
    # gives under the same comparison
    "fp32_all": (("",), ("",)),
    "fp32_all_dref": (("",), ("",)),
}
# the batch-2 'mixed' case of tests/test_configs_gpu.py::test_cfg3_redweb_448 (PLD_EXP_CASE=b2):
# which FFL2 conv carries the error on ffl2/block_down/bn3/gamma
FFL2_DOWN = "ffl2/block_down"
VARIANTS_B2 = {
    "mixed": ((), ()),
    "ffl2_down_fwd": ((FFL2_DOWN,), ()),
    "ffl2_down_bwd": ((), (FFL2_DOWN,)),
    "ffl2_down_fwdbwd": ((FFL2_DOWN,), (FFL2_DOWN,)),
    "ffl2_fwdbwd": (("ffl2",), ("ffl2",)),
    "ffl_fwdbwd": (("ffl",), ("ffl",)),
    "dec_all_fwdbwd": (("ffl", "aol"), ("ffl", "aol")),
}
for _i in range(6):
    _n = f"{FFL2_DOWN}/conv{_i}"
    VARIANTS_B2[f"ffl2_down_conv{_i}_fwdbwd"] = ((_n,), (_n,))
for _n in ("ffl2/conv0", "ffl2/conv1", "ffl2/block_left"):
    VARIANTS_B2[_n.replace("/", "_") + "_fwdbwd"] = ((_n,), (_n,))


def rel(a, b):
    a = torch.as_tensor(a).detach().double().cpu()
    b = torch.as_tensor(b).detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp(min=1e-30))


def _heartbeat():
    import threading

    def beat():
        t0 = time.time()
        while True:
            time.sleep(50)
            print(f"  ... {time.time() - t0:.0f} s", flush=True)
    threading.Thread(target=beat, daemon=True).start()


def _rankings(rng, B, H, R, L):
    idx = rng.integers(0, H * H, (B, R, L))
    lab = rng.permutation(B * R * L).reshape(B, R, L) / (B * R * L)
    lab = -np.sort(-lab, axis=-1)
    return np.ascontiguousarray(np.stack([idx.astype(np.float32), lab.astype(np.float32)], -1))


def main():
    case = os.environ.get("PLD_EXP_CASE", "b32")
    table = VARIANTS if case == "b32" else VARIANTS_B2
    names = sys.argv[1:] or list(table)
    _heartbeat()
    torch.cuda.set_device(0)
    H, R, L = 448, 100, 5
    if case == "b32":
        math = "auto"
        K.set_conv_math(math)
        n_tab, sha = K.use_schedule_table()
        B = 32
        rng = np.random.default_rng(32)
        x = preprocess_input(rng.random((B, H, H, 3)).astype(np.float32))
        y = _rankings(rng, B, H, R, L)
    else:
        # exactly test_cfg3_redweb_448: built-in schedules (fixed_schedules), seed 4
        math, sha, B = "mixed", "builtin", 2
        K.AUTOTUNE = False
        K._TILE_CACHE.clear()
        rng = np.random.default_rng(4)
        x = preprocess_input(rng.random((B, H, H, 3)).astype(np.float32))
        y = _rankings(rng, B, H, R, L)
    eng = RedWebFF((H, H, 3), B, seed=0, conv_math=math)
    W = eng.get_weights()
    P = {k: torch.tensor(v, dtype=torch.float64) for k, v in W.items()}
    P32 = {k: torch.tensor(v, dtype=torch.float32) for k, v in W.items()}
    x64 = torch.tensor(x, dtype=torch.float64)
    zeros = {"aol/conv0/bias", "aol/conv1/bias", "aol/conv2/bias"}
    t0 = time.time()
    b32 = {}
    with torch.no_grad():
        pred_ref = OR.forward(P, x64, preprocessed=True)
        OR.forward(P32, torch.tensor(x), preprocessed=True, relu_branches=b32)
    loss_ref, dpred_ref = LM.hourglass_nll(y, pred_ref.numpy(), B, L)
    dref = torch.tensor(dpred_ref, dtype=torch.float64)
    g32 = OR.train_step_grads(P32, torch.tensor(x), dref.float(), preprocessed=True)[0]
    g64f = OR.train_step_grads(P, x64, dref, preprocessed=True, relu_masks=b32)[0]
    e32 = {k: rel(g32[k], g64f[k]) for k in g64f if k not in zeros}
    # the fp32 restatement end to end: its own forward's dL/dpred
    with torch.no_grad():
        pred32 = OR.forward(P32, torch.tensor(x), preprocessed=True)
    _, dpred32 = LM.hourglass_nll(y, pred32.double().numpy(), B, L)
    g32o = OR.train_step_grads(P32, torch.tensor(x), torch.tensor(dpred32).float(),
                               preprocessed=True)[0]
    e32_own = {k: rel(g32o[k], g64f[k]) for k in g64f if k not in zeros}
    print("fp32 end-to-end within 1e-3:", sum(e <= TOL for e in e32_own.values()),
          "dpred32 vs dref", rel(torch.tensor(dpred32), dref), flush=True)
    del g32, g64f, g32o
    # a second fp32 restatement: torch's native (im2col + sgemm) convolutions instead of oneDNN,
    # i.e. the same semantics with another summation order, along its own ReLU branches
    e32b = {}
    if os.environ.get("PLD_EXP_FP32B", "1") == "1":
        t1 = time.time()
        with torch.backends.mkldnn.flags(enabled=False):
            b32b = {}
            with torch.no_grad():
                OR.forward(P32, torch.tensor(x), preprocessed=True, relu_branches=b32b)
            g32b = OR.train_step_grads(P32, torch.tensor(x), dref.float(), preprocessed=True)[0]
        g64b = OR.train_step_grads(P, x64, dref, preprocessed=True, relu_masks=b32b)[0]
        e32b = {k: rel(g32b[k], g64b[k]) for k in g64b if k not in zeros}
        del g32b, g64b, b32b
        both = sum(max(e32[k], e32b[k]) <= TOL for k in e32)
        print(f"second fp32 restatement (no oneDNN): within 1e-3 {sum(e <= TOL for e in e32b.values())}"
              f", both within {both} ({time.time() - t1:.0f} s)", flush=True)
    print(f"reference + fp32 restatement: {time.time() - t0:.0f} s", flush=True)
    out = {"schedule_table": sha, "fp32_restatement": e32, "fp32_restatement_own_dpred": e32_own,
           "fp32_restatement_native_conv": e32b, "variants": {}}
    yt = torch.from_numpy(y).cuda()
    for v in names:
        fwd, bwd = table[v]
        eng.exact_fwd_extra, eng.exact_bwd = fwd, bwd
        eng.set_weights(W)
        eng.act["input"].copy_(torch.from_numpy(x))
        pred = eng.forward(training=True)
        mr = {st: (eng.act[st] > 0).permute(0, 3, 1, 2).cpu() for st in OR.relu_sites()}
        loss, dpred, _ = K.listmle_fwd_bwd(pred, yt, B, R, L)
        e_dpred = rel(dpred, dref)
        if v.endswith("_dref"):
            dpred = dref.float().to(pred.device).reshape(dpred.shape)
        eng.backward(dpred)
        torch.cuda.synchronize()
        e_pred = rel(pred, pred_ref)
        hip = {k: eng.grads[k].detach().cpu() for k in e32}
        # eager fwd+bwd time (schedules fixed by the table)
        t1 = time.time()
        for _ in range(3):
            eng.forward(training=True)
            eng.backward(dpred)
        torch.cuda.synchronize()
        ms = (time.time() - t1) / 3 * 1e3
        t1 = time.time()
        g64h = OR.train_step_grads(P, x64, dref, preprocessed=True, relu_masks=mr)[0]
        eh = {k: rel(hip[k], g64h[k]) for k in e32}
        del g64h
        strict_fail = {k: (eh[k], e32[k]) for k in e32 if e32[k] <= TOL and eh[k] > TOL}
        if e32b:
            # the round-6 bar: against the worse of the two fp32 restatements
            worse = {k: max(e32[k], e32b[k]) for k in e32}
            ratio = sorted(((eh[k] / max(worse[k], 1e-30), k, eh[k], e32[k], e32b[k])
                            for k in e32 if eh[k] > TOL), reverse=True)[:8]
            print(f"  {v}: HIP/worse-fp32 over 1e-3: " + ", ".join(
                f"{k} {r:.2f} ({a:.2e} vs {b:.2e}/{c:.2e})" for r, k, a, b, c in ratio), flush=True)
        loose_fail = {k: (eh[k], e32[k]) for k in e32 if e32[k] > TOL and eh[k] > 2 * e32[k]}
        worst = sorted(eh.items(), key=lambda kv: -kv[1] / max(e32[kv[0]], TOL))[:12]
        out["variants"][v] = {"exact_fwd": fwd, "exact_bwd": bwd, "ms_fwd_bwd": ms,
                              "pred": e_pred, "dpred": e_dpred, "within_1e-3": sum(e <= TOL for e in eh.values()),
                              "tensors": len(eh), "strict_fail": strict_fail,
                              "loose_fail": loose_fail, "worst": worst, "errors": eh}
        print(f"{v}: {ms:.1f} ms  pred {e_pred:.2e}  dpred {e_dpred:.2e}  within {out['variants'][v]['within_1e-3']}"
              f"/{len(eh)}  strict_fail {len(strict_fail)} {sorted(strict_fail.items())[:6]}  "
              f"loose_fail {len(loose_fail)}  (oracle {time.time() - t1:.0f} s)", flush=True)
        os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
        with open(os.path.join(ROOT, "gpurun_out", f"redweb_parity_{case}.json"), "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
