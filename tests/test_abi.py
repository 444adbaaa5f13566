"""CPU tests of the C ABI boundary: the library loads and exports every declared symbol."""
import ctypes as C
import os
import subprocess

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


def test_header_documents_reference_replacements():
    txt = open(_lib.HEADER).read()
    for ref in ["depth_utils.py:39-61", "nll_loss.py", "PLDepth.py:133", "pl_hourglass.py",
                "sampling.py"]:
        assert ref in txt, ref
