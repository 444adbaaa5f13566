"""CPU tests of the C ABI boundary: the library loads and exports every declared symbol."""
import ctypes as C
import os
import subprocess

import pytest

from pldepth_amd import _lib


def test_library_exports_every_declared_symbol():
    lib = _lib.lib()
    declared = _lib.declared_symbols()
    assert len(declared) >= 30
    missing = [s for s in declared if not hasattr(lib._dll, s)]
    assert not missing, missing
    # every declared symbol has a ctypes signature, and vice versa
    assert set(declared) == set(_lib._SIGS), set(declared) ^ set(_lib._SIGS)


def test_exports_are_plain_c_symbols():
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if " T " in ln}
    for s in _lib.declared_symbols():
        assert s in exported, s  # unmangled extern "C"


def test_host_only_entry_points():
    lib = _lib.lib()
    assert lib.pld_version() == 1
    assert lib.pld_sampler_candidates(100, 3) == 500
    assert lib.pld_sampler_candidates(100, 0) == 80
    assert lib.pld_sampler_candidates(100, 2) == 150
    # argument validation fails loudly before touching the GPU
    try:
        lib.pld_listmle_fwd_bwd(None, None, 1, 1, 1, 1, None, None, None, 1, None)
    except _lib.PLDError as e:
        assert "null pointer" in str(e)
    else:
        raise AssertionError("expected PLDError")
    a = _lib.ConvArgs()
    assert lib.pld_conv2d_wgrad_workspace_size(C.byref(a)) == 0  # invalid geometry
    assert lib.pld_conv2d_fwd_workspace_size(C.byref(a)) == 0
    assert lib.pld_conv2d_dgrad_workspace_size(C.byref(a)) == 0
    # split-K schedules of a deep, small-M GEMM need a slab workspace; plain ones do not
    a.n, a.h, a.w, a.c1, a.kh, a.kw, a.sh, a.sw = 1, 7, 7, 1024, 3, 3, 1, 1
    a.pad_t = a.pad_l = 1
    a.oh, a.ow, a.cout = 7, 7, 64
    nt = lib.pld_conv_num_tiles()
    a.tile = 0
    assert lib.pld_conv2d_fwd_workspace_size(C.byref(a)) == 0
    a.tile = nt // 2
    assert lib.pld_conv2d_fwd_workspace_size(C.byref(a)) >= 2 * 49 * 64 * 4


def test_filter_refresh_plan_and_descriptor_layout():
    """pld_filter_refresh_plan (host arithmetic only): the block count of a filter's batched
    refresh, 0 where the batched path does not apply; the ctypes descriptor matches the
    header's pld_filter_refresh_desc (5 pointers + 6 ints = 64 B)."""
    from pldepth_amd import kernels as K
    lib = _lib.lib()
    p, q = C.c_void_p(1 << 20), C.c_void_p((1 << 20) + 4)  # 16-byte aligned / not
    # 3x3, 64 -> 64: 9 x 1 native tiles + ceil(576 * 64 / 8 / 256) = 18 dgrad blocks
    assert lib.pld_filter_refresh_plan(3, 3, 64, 64, p, p, p, p, p) == 9 + 18
    assert lib.pld_filter_refresh_plan(3, 3, 64, 64, p, p, None, None, None) == 9
    assert lib.pld_filter_refresh_plan(3, 3, 3, 32, p, p, p, p, p) == 0   # R = 27 % 8
    assert lib.pld_filter_refresh_plan(3, 3, 64, 100, p, p, p, p, p) == 0  # dgrad cout % 8
    assert lib.pld_filter_refresh_plan(3, 3, 64, 64, p, q, p, p, p) == 0   # misaligned
    assert lib.pld_filter_refresh_plan(3, 3, 64, 64, p, p, p, None, p) == 0  # split w/o dgrad
    assert C.sizeof(K._RefreshDesc) == 64
    with pytest.raises(_lib.PLDError):
        lib.pld_filter_refresh_multi(None, 1, 1, None)


def test_header_documents_reference_replacements():
    txt = open(_lib.HEADER).read()
    for ref in ["depth_utils.py:39-61", "nll_loss.py", "PLDepth.py:133", "pl_hourglass.py",
                "sampling.py"]:
        assert ref in txt, ref


def test_schedule_names_are_unique_and_resolve():
    """pld_conv_schedule_desc names every schedule once per math; the persisted table
    (kernels.DEFAULT_SCHEDULES) names only schedules this build has, for gfx950."""
    import json

    from pldepth_amd import kernels as K
    lib = _lib.lib()
    for math in K.MATH.values():
        n = lib.pld_conv_num_schedules(math)
        names = [lib.pld_conv_schedule_desc(math, i).decode() for i in range(n)]
        assert len(set(names)) == n, names
        assert lib.pld_conv_schedule_desc(math, n) is None
        assert all(K._schedule_index(math, d) == i for i, d in enumerate(names))
    if os.path.exists(K.DEFAULT_SCHEDULES):
        d = json.load(open(K.DEFAULT_SCHEDULES))
        assert d["format"] == K.SCHEDULE_FORMAT and d["arch"].startswith("gfx950")
        assert d["entries"]
        for key, desc in d["entries"]:
            assert len(key) == len(d["key"])
            assert K._schedule_index(key[-1], desc) is not None, (key, desc)
        # the same entries are taken on a gfx950 device (arch given: no GPU here)
        saved = dict(K._TILE_CACHE)
        try:
            K._TILE_CACHE.clear()
            assert K.load_tile_cache(K.DEFAULT_SCHEDULES, arch=d["arch"]) == len(d["entries"])
        finally:
            K._TILE_CACHE.clear()
            K._TILE_CACHE.update(saved)


def test_bench_self_spawn_command(monkeypatch):
    """bench.py --gpus N without a launcher runs torch.distributed.run with N ranks on
    127.0.0.1 as one child process and exits with its code (no GPU call in the parent)."""
    import subprocess as sp
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    seen = {}

    def fake_call(cmd, env=None):
        seen["cmd"], seen["env"] = cmd, env
        return 7

    monkeypatch.setattr(sp, "call", fake_call)
    assert bench.spawn_ranks(8, ["--gpus", "8", "--steps", "3"]) == 7
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert cmd[cmd.index("--nproc-per-node") + 1] == "8"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "8", "--steps", "3"] and cmd[-5].endswith("bench.py")
