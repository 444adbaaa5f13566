"""Time the ROCm library GEMM (torch.matmul: hipBLASLt / rocBLAS) on the short-M 1x1 conv GEMM
shapes, bf16 and fp32, from replayed CUDA graphs — the reference point for the bf16x3 1x1 launches
(profiles/r06_short_m_library_floor.txt). python tools/gemm_library_floor.py"""
import torch, time
torch.cuda.set_device(0)
def t(f, n=50):
    f(); torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        f(); s.synchronize()
        with torch.cuda.graph(g, stream=s):
            for _ in range(10): f()
    g.replay(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n): g.replay()
    e1.record(); e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (10 * n)
for (M, K, N) in [(6272, 1152, 192), (6272, 192, 1152), (25088, 480, 80), (1568, 1152, 192), (6272, 64, 64)]:
    for dt in (torch.bfloat16, torch.float32):
        a = torch.randn(M, K, device="cuda", dtype=dt); b = torch.randn(K, N, device="cuda", dtype=dt)
        c = torch.empty(M, N, device="cuda", dtype=dt)
        us = t(lambda: torch.matmul(a, b, out=c))
        print(f"M{M} K{K} N{N} {dt}: {us:.2f} us  {2*M*K*N/us/1e6:.1f} TF/s", flush=True)
x = torch.empty(1, device="cuda")
print("empty kernel (fill_):", f"{t(lambda: x.fill_(1.0)):.2f} us")
