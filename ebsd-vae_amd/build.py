"""Build libebsdvae.so (all HIP kernels + the C ABI of include/ebsdvae.h) for gfx950.

Plain hipcc, in-tree output (ebsd-vae_amd/lib/libebsdvae.so) so the library travels with
the repo snapshot to the GPU box.  Incremental: an object is rebuilt only when its source,
a csrc header or the public header is newer.

    python ebsd-vae_amd/build.py [-j N] [--force]
    python ebsd-vae_amd/build.py --variant NAME -D FLAG ...   # experiment build (A/B timing):
        lib/libebsdvae_NAME.so with -DFLAG..., selected at run time by EBSDVAE_LIB=<path>
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(HERE, "build")
LIB_DIR = os.path.join(HERE, "lib")
LIB = os.path.join(LIB_DIR, "libebsdvae.so")
HEADER = os.path.join(REPO, "include", "ebsdvae.h")
ARCH = os.environ.get("EBSDVAE_ARCH", "gfx950")


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm toolchain required to build libebsdvae.so)")


def sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip"))


def _stale(src: str, obj: str) -> bool:
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    deps = [src, HEADER] + [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    return any(os.path.getmtime(d) > t for d in deps)


# host-only AddressSanitizer flags: each -fsanitize= directly after -Xarch_host, so the device
# code is built as usual (GPU ASan is not used)
ASAN_HOST = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fno-omit-frame-pointer"]


def _compile(src: str, force: bool, objdir: str = OBJ, defines=(), extra=()) -> str:
    obj = os.path.join(objdir, os.path.basename(src) + ".o")
    if force or _stale(src, obj):
        cmd = [_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
               "-Wall", "-Wno-unused-function"] + list(extra) + [f"-D{d}" for d in defines] + \
              ["-c", src, "-o", obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
    return obj


def build(jobs: int = 8, force: bool = False, verbose: bool = True, variant: str = "",
          defines=()) -> str:
    objdir = OBJ if not variant else os.path.join(OBJ, variant)
    lib = LIB if not variant else os.path.join(LIB_DIR, f"libebsdvae_{variant}.so")
    os.makedirs(objdir, exist_ok=True)
    os.makedirs(LIB_DIR, exist_ok=True)
    srcs = sources()
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        objs = list(ex.map(lambda s: _compile(s, force or bool(variant), objdir, defines), srcs))
    LIB_ = lib
    if force or not os.path.exists(LIB_) or any(os.path.getmtime(o) > os.path.getmtime(LIB_) for o in objs):
        tmp = LIB_ + ".tmp"
        cmd = [_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, LIB_)
    if verbose:
        print(f"built {LIB_}")
    return LIB_


def build_asan(jobs: int = 8, verbose: bool = True) -> str:
    """Host-ASan build of the library objects linked into tests/asan/abi_asan.cpp, a driver
    of the C ABI's argument validation, scratch-size queries and error plumbing (no GPU
    needed).  Output: ebsd-vae_amd/build/asan/abi_asan (run by tests/test_abi.py)."""
    objdir = os.path.join(OBJ, "asan")
    os.makedirs(objdir, exist_ok=True)
    drv = os.path.join(REPO, "tests", "asan", "abi_asan.cpp")
    srcs = sources()
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        objs = list(ex.map(lambda s: _compile(s, False, objdir, extra=ASAN_HOST + ["-g"]), srcs))
    exe = os.path.join(objdir, "abi_asan")
    if not os.path.exists(exe) or any(os.path.getmtime(d) > os.path.getmtime(exe)
                                      for d in objs + [drv, HEADER]):
        cmd = [_hipcc(), f"--offload-arch={ARCH}", "-O1", "-g", "-std=c++17", "-x", "c++", drv,
               "-x", "none"] + objs + ASAN_HOST + ["-fsanitize=address", "-o", exe + ".tmp"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"asan link failed:\n{r.stdout}\n{r.stderr}")
        os.replace(exe + ".tmp", exe)
    if verbose:
        print(f"built {exe}")
    return exe


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--variant", default="")
    ap.add_argument("-D", dest="defines", action="append", default=[])
    ap.add_argument("--asan", action="store_true", help="host-ASan C-ABI driver (tests/asan)")
    a = ap.parse_args()
    if a.asan:
        build_asan(a.j)
        return
    build(a.j, a.force, variant=a.variant, defines=a.defines)


if __name__ == "__main__":
    sys.exit(main())
