"""Per-call timing table of the BatchNorm passes of one training step (HIP events around every
BN entry point), with each call's floor bytes (every distinct tensor it is handed read or
written once) and the rate that implies.

    python tools/bn_table.py [--model ff_redweb] [--size 448] [--batch 32] [--top 40]

One eager step tunes the conv schedules, a second eager step is timed call by call.
"""
import argparse
import collections
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# floor bytes per element: tensors read + written once
FLOOR = {"bn_apply": 8, "bn_add_apply": 12, "bn_bwd": 12, "bn_add_bwd": 20, "bn_stats": 4,
         "bn_bwd_coeffs": 8}


def timed_step(tr, lr):
    from pldepth_amd import kernels as K
    st = tr.stream
    recs = []
    orig = {n: getattr(K, n) for n in FLOOR}

    def wrap(name):
        fn = orig[name]

        def w(x, *rest, **kw):
            rows, c = rest[0], rest[1]
            if name == "bn_bwd" or name == "bn_add_bwd" or name == "bn_bwd_coeffs":
                rows, c = rest[1], rest[2]
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            r = fn(x, *rest, **kw)
            e1.record(st)
            recs.append((name, int(rows), int(c), e0, e1))
            return r
        return w

    for n in orig:
        setattr(K, n, wrap(n))
    overlap = getattr(tr.engine, "overlap_wgrad", False)
    tr.engine.overlap_wgrad = False  # one stream: the events bracket each call alone
    try:
        tr.step_eager(lr)
        st.synchronize()
    finally:
        tr.engine.overlap_wgrad = overlap
        for n, f in orig.items():
            setattr(K, n, f)
    return [(n, r, c, e0.elapsed_time(e1)) for n, r, c, e0, e1 in recs]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="ff_redweb")
    ap.add_argument("--size", type=int, default=448)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    import bench
    from pldepth_amd.trainer import ReplicaTrainer
    torch.cuda.set_device(0)
    H = a.size
    tr = ReplicaTrainer((H, H, 3), a.batch, 5, 100, 1, seed=0, model=a.model)
    x, gt, mask = bench.synthetic_batch(a.batch, H, H, seed=1000)
    if a.model == "ff_redweb":
        x = tr.engine.preprocess(x)
    tr.set_batch(torch.from_numpy(x).cuda(), torch.from_numpy(gt).cuda(),
                 torch.from_numpy(mask).cuda())
    tr.step_eager(0.01)  # tunes
    torch.cuda.synchronize()
    recs = timed_step(tr, 0.01)
    print(f"{'op':14} {'rows':>9} {'c':>5} {'ms':>7} {'floorGB':>8} {'GB/s':>7}")
    for n, r, c, ms in sorted(recs, key=lambda t: -t[3])[:a.top]:
        gb = FLOOR[n] * r * c / 1e9
        print(f"{n:14} {r:9d} {c:5d} {ms:7.3f} {gb:8.3f} {gb / ms * 1e3:7.0f}")
    agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
    for n, r, c, ms in recs:
        agg[n][0] += 1
        agg[n][1] += ms
        agg[n][2] += FLOOR[n] * r * c / 1e9
    tot = sum(v[1] for v in agg.values())
    for n, (cnt, ms, gb) in sorted(agg.items(), key=lambda t: -t[1][1]):
        print(f"{n}: {cnt} calls {ms:.3f} ms, floor {gb:.2f} GB -> {gb / ms * 1e3:.0f} GB/s")
    print(f"BN total {tot:.3f} ms over {len(recs)} calls")


if __name__ == "__main__":
    main()
