"""Per-conv timing table of one training step (HIP events around every conv launch).

    python tools/conv_table.py [--model ff_effnet] [--size 448] [--batch 32]
                               [--math bf16x3 fp32] [--top 40]

For each conv math: one eager step tunes every shape's schedule, a second eager step is timed
conv by conv. Rows are matched across maths by call order (same step, same shapes).
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def a_pro(args):
    return bool(args.in_scale)


def timed_step(tr, lr):
    from pldepth_amd import kernels as K
    st = tr.stream
    recs = []
    orig = {n: getattr(K, n) for n in ("conv2d_fwd", "conv2d_dgrad", "conv2d_wgrad",
                                       "conv2d_fwd_bn_stats")}

    def wrap(name):
        fn = orig[name]

        def w(args, *rest, **kw):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            r = fn(args, *rest, **kw)
            e1.record(st)
            mode = name.split("_")[1]
            if a_pro(args):
                mode += "+p"
            if mode.startswith("fwd"):
                M, N, Kd = args.n * args.oh * args.ow, args.cout, args.kh * args.kw * (args.c1 + args.c2)
            elif mode == "dgrad":
                M, N, Kd = args.n * args.h * args.w, args.c1 + args.c2, args.kh * args.kw * args.cout
            else:
                M, N, Kd = args.kh * args.kw * (args.c1 + args.c2), args.cout, args.n * args.oh * args.ow
            saved = args.tile
            args.tile = getattr(args, "_used_tile", saved)
            kname = K.conv_kernel_name(args, mode.split("+")[0] if mode != "fwd_bn_stats"
                                       else "fwd")
            sched = K.schedule_desc(args.math, args.tile)
            args.tile = saved
            by = 4.0 * (args.n * args.h * args.w * (args.c1 + args.c2)
                        + args.n * args.oh * args.ow * args.cout
                        + args.kh * args.kw * (args.c1 + args.c2) * args.cout)
            recs.append((mode, M, N, Kd, args.kh, (kname, sched, by), e0, e1))
            return r
        return w

    for n in orig:
        setattr(K, n, wrap(n))
    overlap = getattr(tr.engine, "overlap_wgrad", False)
    tr.engine.overlap_wgrad = False  # one stream: the events bracket each conv alone
    try:
        tr.step_eager(lr)
        st.synchronize()
    finally:
        tr.engine.overlap_wgrad = overlap
        for n, f in orig.items():
            setattr(K, n, f)
    return [(m, M, N, Kd, k, t, e0.elapsed_time(e1)) for m, M, N, Kd, k, t, e0, e1 in recs]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="ff_effnet")
    ap.add_argument("--size", type=int, default=448)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--math", nargs="+", default=["auto", "mixed", "fp32"])
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--schedules", default="",
                    help="persisted schedule table (kernels.use_schedule_table): no tuning")
    a = ap.parse_args()
    import bench
    from pldepth_amd import kernels as K
    from pldepth_amd.trainer import ReplicaTrainer
    torch.cuda.set_device(0)
    if a.schedules:
        print("schedule table entries:", K.use_schedule_table(a.schedules)[0])
    H = a.size
    tr = ReplicaTrainer((H, H, 3), a.batch, 5, 100, 1, seed=0, model=a.model)
    x, gt, mask = bench.synthetic_batch(a.batch, H, H, seed=1000)
    if a.model == "ff_redweb":
        x = tr.engine.preprocess(x)
    tr.set_batch(torch.from_numpy(x).cuda(), torch.from_numpy(gt).cuda(),
                 torch.from_numpy(mask).cuda())
    tables = {}
    for m in a.math:
        tr.engine.enc_math, tr.engine.dec_math = K.conv_policy(m)
        tr.step_eager(0.01)  # tunes
        torch.cuda.synchronize()
        tables[m] = timed_step(tr, 0.01)
    base = tables[a.math[0]]
    order = sorted(range(len(base)), key=lambda i: -base[i][6])
    hdr = "  ".join(f"{m:>16}" for m in a.math)
    print(f"{'mode':6} {'M':>9} {'N':>5} {'K':>8} k  {hdr}   kernel / schedule / GB/s")
    for i in order[:a.top]:
        mode, M, N, Kd, k, (kname, sched, by), _ = base[i]
        fl = 2.0 * M * N * Kd
        cells = "  ".join(f"{tables[m][i][6]:7.3f}ms {fl / tables[m][i][6] / 1e9:5.0f}TF"
                          for m in a.math)
        print(f"{mode:6} {M:9d} {N:5d} {Kd:8d} {k}  {cells}   {kname} {sched} "
              f"{by / base[i][6] / 1e6:6.0f}")
    for m in a.math:
        tot = sum(r[6] for r in tables[m])
        fl = sum(2.0 * r[1] * r[2] * r[3] for r in tables[m])
        print(f"{m}: total conv {tot:.3f} ms over {len(tables[m])} launches, "
              f"{fl / tot / 1e9:.1f} TF/s")


if __name__ == "__main__":
    main()
