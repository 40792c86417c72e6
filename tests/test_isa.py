"""Static checks of the built gfx950 code (CPU; reads libhdverify.so).

No kernel of the library may contain a device function call (s_swappc).  A
call makes the kernel keep call frames and callee-saved spills next to its
own spill slots; the full recovery emitted as a called function computed
wrong points on gfx950 while every inlined build of the same code matched the
host bit for bit (scripts/w4_probe.hip), and the 4-wave k_verify
that once returned SIGNATORY_MISMATCH for every VALID message called the
out-of-line doubling (gej_dbl_slow, now inlined).  This test keeps the
library call-free.  (s_getpc / s_setpc pairs without s_swappc are the long
branches of a large kernel, not calls.)"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "hyperdrive_amd", "_lib", "libhdverify.so")
LLVM = "/opt/rocm/lib/llvm/bin"
BUNDLER = os.path.join(LLVM, "clang-offload-bundler")
OBJDUMP = os.path.join(LLVM, "llvm-objdump")


def _code_objects(tmp_path):
    data = open(LIB, "rb").read()
    fat = tmp_path / "fatbin.bin"
    subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", LIB, str(fat)], check=True)
    data = fat.read_bytes()
    offs = [m.start() for m in re.finditer(re.escape(b"__CLANG_OFFLOAD_BUNDLE__"), data)] + [len(data)]
    out = []
    for k in range(len(offs) - 1):
        b = tmp_path / f"b{k}.bin"
        co = tmp_path / f"b{k}.co"
        b.write_bytes(data[offs[k]:offs[k + 1]])
        r = subprocess.run([BUNDLER, "--unbundle", "--type=o", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                            f"--input={b}", f"--output={co}"], capture_output=True, text=True)
        if r.returncode == 0 and co.stat().st_size:
            out.append(co)
    return out


@pytest.mark.skipif(not (os.path.exists(LIB) and os.path.exists(BUNDLER) and os.path.exists(OBJDUMP)
                         and shutil.which("objcopy")), reason="library or ROCm binutils absent")
def test_no_device_calls_in_kernels(tmp_path):
    cos = _code_objects(tmp_path)
    assert len(cos) >= 5                              # one code object per .hip translation unit
    calls, kernels = {}, set()
    for co in cos:
        d = subprocess.run([OBJDUMP, "-d", str(co)], capture_output=True, text=True, check=True).stdout
        cur = None
        for line in d.splitlines():
            m = re.match(r"^[0-9a-f]+ <(.*)>:$", line)
            if m:
                cur = m.group(1)
                kernels.add(cur)
                continue
            if "s_swappc" in line:           # (s_setpc alone is a long branch in a big kernel)
                calls[cur] = calls.get(cur, 0) + 1
    assert any("k_verify" in k for k in kernels) and any("k_fast_sums" in k for k in kernels)
    assert calls == {}, calls
