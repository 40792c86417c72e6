"""Build the in-tree native library ``hyperdrive_amd/_lib/libhdverify.so``.

Each ``csrc/*.hip`` / ``csrc/*.cpp`` translation unit is compiled for gfx950 in parallel with
``hipcc -c`` and linked with ``hipcc -shared``.  The library is built in-tree
so that it travels with the repository snapshot to the GPU box.

Usage: ``python -m hyperdrive_amd.build [--force] [--jobs N]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "_lib")
OBJDIR = os.environ.get("HD_BUILD_OBJDIR", os.path.join(LIBDIR, "obj"))
LIB = os.environ.get("HD_BUILD_LIB", os.path.join(LIBDIR, "libhdverify.so"))
INCLUDE = os.path.join(os.path.dirname(HERE), "include")
ARCH = os.environ.get("HD_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", shutil.which("hipcc") or "/opt/rocm/bin/hipcc")
ROCM_LIB = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "lib")

CFLAGS = ["--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function",
          "-I" + INCLUDE] + ["-D%s=%s" % (k, os.environ[k]) for k in ("HD_FB_W", "HD_FB_WG") if os.environ.get(k)] \
    + os.environ.get("HD_EXTRA_CFLAGS", "").split()   # A/B builds (e.g. into HD_BUILD_LIB under _lib/var/)


def _sources():
    # *.hip: device + host code; *.cpp: host-only C++ (hd_votes)
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))


def _deps():
    return (sorted(glob.glob(os.path.join(CSRC, "*.h"))) + sorted(glob.glob(os.path.join(INCLUDE, "*.h")))
            + [os.path.abspath(__file__)])


def _mtime(p):
    try:
        return os.path.getmtime(p)
    except OSError:
        return -1.0


def _compile(src: str, force: bool):
    """(object path, whether it was compiled now)"""
    obj = os.path.join(OBJDIR, os.path.basename(src) + ".o")
    newest = max([_mtime(src)] + [_mtime(d) for d in _deps()])
    if not force and _mtime(obj) >= newest:
        return obj, False
    cmd = [HIPCC, *CFLAGS, "-c", src, "-o", obj]
    t0 = time.time()
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr[-6000:]}")
    # the object is as old as the sources it was compiled from: a source
    # edited while hipcc ran is newer than it, so the next build recompiles
    os.utime(obj, (t0, t0))
    return obj, True


def build(force: bool = False, jobs: int | None = None, verbose: bool = True) -> str:
    """Compile every HIP translation unit and link libhdverify.so."""
    os.makedirs(OBJDIR, exist_ok=True)
    srcs = _sources()
    jobs = jobs or min(len(srcs), max(1, (os.cpu_count() or 4)))
    jobs = min(jobs, 16)
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        done = list(ex.map(lambda s: _compile(s, force), srcs))
    objs = [o for o, _ in done]
    if force or any(c for _, c in done) or _mtime(LIB) < max(_mtime(o) for o in objs):
        tmp = LIB + ".tmp"
        # librccl: the hd_multi_* exchange (hd_multi.hip)
        r = subprocess.run([HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC", *objs, "-L" + ROCM_LIB, "-lrccl",
                            "-Wl,-rpath," + ROCM_LIB, "-o", tmp],
                           capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr[-4000:]}")
        os.replace(tmp, LIB)
        if verbose:
            print(f"[hyperdrive_amd] built {LIB}", file=sys.stderr)
    return LIB


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=None)
    a = ap.parse_args()
    build(force=a.force, jobs=a.jobs)
