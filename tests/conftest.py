"""Shared fixtures.

* ``gpu`` marker: tests that need an MI355X (run with ``-m gpu``).
* ``oracle``: the pure-Python restatement (oracle/hd_pyoracle.py).
* ``coracle``: the C restatement (oracle/hd_oracle.c -> oracle/_build/liboracle.so).
* ``hostmath``: a host (g++) build of the device math headers -- the exact
  arithmetic the kernels run, exercised on CPU (tests/native/hd_host_check.cpp).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
NATIVE_DIR = os.path.join(ROOT, "tests", "native")
sys.path.insert(0, ROOT)
sys.path.insert(0, ORACLE_DIR)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD MI355X GPU (run with -m gpu)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def _newer(target, sources):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in sources)


def build_coracle() -> str:
    out = os.path.join(ORACLE_DIR, "_build", "liboracle.so")
    src = [os.path.join(ORACLE_DIR, "hd_oracle.c"), os.path.join(ORACLE_DIR, "Makefile")]
    if _newer(out, src):
        subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)
    return out


def build_hostmath(bounds: bool = False) -> str:
    """bounds=True builds with -DHD_BOUNDS: every field element then carries
    interval bounds that each operation checks (hd_field.h).  With
    HD_HOST_SANITIZE=1 in the environment the build adds UBSan
    (-fsanitize=undefined, any finding aborts), so the host-math suite runs
    the device headers under the sanitizer.  HD_HOST_SANITIZE=asan adds
    AddressSanitizer as well; the interpreter then needs the ASan runtime
    preloaded:
        LD_PRELOAD=$(gcc -print-file-name=libasan.so) ASAN_OPTIONS=detect_leaks=0 \
        HD_HOST_SANITIZE=asan python -m pytest tests -m "not gpu" -k <host-math tests>"""
    mode = os.environ.get("HD_HOST_SANITIZE", "")
    san = mode in ("1", "asan")
    name = ("libhdhost_bounds" if bounds else "libhdhost") + {"1": "_ubsan", "asan": "_asan"}.get(mode, "") + ".so"
    out = os.path.join(NATIVE_DIR, "_build", name)
    csrc = os.path.join(ROOT, "hyperdrive_amd", "csrc")
    srcs = [os.path.join(NATIVE_DIR, "hd_host_check.cpp")] + [os.path.join(csrc, f) for f in os.listdir(csrc)
                                                              if f.endswith(".h")]
    if _newer(out, srcs):
        os.makedirs(os.path.dirname(out), exist_ok=True)
        # the fixed-base tables at 12-bit windows (22 x 2048 entries): the
        # product's 16-bit tables (17 x 32768) take ~10 s per key to build on
        # one host core; the algorithm is the same for every window width
        flags = (["-DHD_BOUNDS"] if bounds else []) + ["-DHD_FB_W=12", "-DHD_FB_WG=12"]
        if san:
            flags += ["-fsanitize=undefined", "-fno-sanitize-recover=all", "-g"]
        if mode == "asan":
            flags += ["-fsanitize=address", "-fno-omit-frame-pointer"]
        subprocess.run(["g++", "-O2", "-fPIC", "-shared", "-std=c++17", "-Wall", "-Wno-unused-function", *flags, "-o",
                        out, srcs[0]], check=True)
    return out


@pytest.fixture(scope="session")
def oracle():
    import hd_pyoracle
    return hd_pyoracle


@pytest.fixture(scope="session")
def coracle():
    from oracle_c import COracle
    return COracle(build_coracle())


@pytest.fixture(scope="session")
def hostmath():
    from hostmath import HostMath
    return HostMath(build_hostmath())


@pytest.fixture(scope="session")
def hostmath_bounds():
    from hostmath import HostMath
    return HostMath(build_hostmath(bounds=True))


@pytest.fixture(scope="session")
def keys(oracle):
    return oracle.KeyCache()


def _gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu():
    if not _gpu_available():
        pytest.fail("GPU test selected but no GPU is visible")
    import hyperdrive_amd as hd
    from hyperdrive_amd import _lib
    _lib.load()  # fails loudly if the HIP library is missing
    return hd
