"""Build libpldepth_hip.so (in-tree) from pldepth_amd/csrc/*.hip for gfx950.

    python -m pldepth_amd.build [--force] [-j N]

One object per source, compiled in parallel with hipcc, linked into
``pldepth_amd/libpldepth_hip.so``. Objects are rebuilt when their source or any header is newer.
"""
import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
BUILD = os.path.join(ROOT, "build", "hip")
LIB = os.path.join(PKG, "libpldepth_hip.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("PLD_OFFLOAD_ARCH", "gfx950")

CFLAGS = [
    f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-Wall", "-Wno-unused-function",
    "-Wno-unused-variable", "-munsafe-fp-atomics", f"-I{os.path.join(ROOT, 'include')}",
]
# sources whose float arithmetic must follow the reference's rounding step by step
NO_CONTRACT = {"sampler.hip"}


def _headers():
    return glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(ROOT, "include", "*.h"))


def _compile(src, force):
    obj = os.path.join(BUILD, os.path.basename(src) + ".o")
    hdr_mtime = max([os.path.getmtime(h) for h in _headers()] + [0])
    if (not force and os.path.exists(obj)
            and os.path.getmtime(obj) >= max(os.path.getmtime(src), hdr_mtime)):
        return obj, None
    flags = list(CFLAGS)
    if os.path.basename(src) in NO_CONTRACT:
        flags.append("-ffp-contract=off")
    cmd = [HIPCC] + flags + ["-c", src, "-o", obj]
    p = subprocess.run(cmd, capture_output=True, text=True)
    if p.returncode != 0:
        return obj, f"$ {' '.join(cmd)}\n{p.stdout}\n{p.stderr}"
    return obj, None


def build(force=False, jobs=8, verbose=True):
    os.makedirs(BUILD, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    if not srcs:
        raise RuntimeError("no HIP sources found in " + CSRC)
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        results = list(ex.map(lambda s: _compile(s, force), srcs))
    errs = [e for _, e in results if e]
    if errs:
        raise RuntimeError("hipcc failed:\n" + "\n".join(errs))
    objs = [o for o, _ in results]
    newest = max(os.path.getmtime(o) for o in objs)
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < newest:
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB] + objs
        p = subprocess.run(cmd, capture_output=True, text=True)
        if p.returncode != 0:
            raise RuntimeError(f"link failed:\n$ {' '.join(cmd)}\n{p.stdout}\n{p.stderr}")
        if verbose:
            print(f"[pldepth_amd.build] linked {LIB} ({len(objs)} objects)")
    elif verbose:
        print(f"[pldepth_amd.build] {LIB} up to date")
    return LIB


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=8)
    a = ap.parse_args(argv)
    build(force=a.force, jobs=a.j)


if __name__ == "__main__":
    sys.exit(main())
