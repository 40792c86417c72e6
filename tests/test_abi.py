"""The C-ABI library loads (no GPU needed) and exports every function that
include/*.h declares; the ctypes binding covers exactly that surface; no
compute is called here."""
import ctypes
import glob
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"^[A-Za-z_][\w\s\*]*?\b(hd_\w+)\s*\(", src, flags=re.M):
            names.add(m.group(1))
    return names


def _lib_path():
    from hyperdrive_amd import build
    if not os.path.exists(build.LIB):
        build.build()
    return build.LIB


def test_headers_declare_the_boundary():
    names = declared_functions()
    for must in ["hd_ctx_create", "hd_ctx_destroy", "hd_set_signatories", "hd_verify_batch",
                 "hd_verify_batch_device", "hd_tally", "hd_tally_device", "hd_process_batch", "hd_strerror",
                 "hd_gen_keys", "hd_gen_batch_device", "hd_probe_valu"]:
        assert must in names


def test_library_exports_every_declared_symbol():
    path = _lib_path()
    lib = ctypes.CDLL(path)
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    assert declared_functions() <= exported


def test_binding_covers_the_header():
    from hyperdrive_amd import _lib
    assert set(_lib.SIGNATURES) == declared_functions()


def test_strerror_without_gpu():
    from hyperdrive_amd import _lib
    lib = _lib.load(_lib_path())
    assert lib.hd_strerror(0) == b"ok"
    assert lib.hd_strerror(-1) == b"invalid argument"
    assert lib.hd_strerror(-4) == b"tally capacity too small"
    assert lib.hd_abi_version() == 2
    # NULL arguments are rejected before any device work
    assert lib.hd_ctx_create(0, None) == -1
    assert lib.hd_verify_batch(None, None, None, None, None) == -1
    assert lib.hd_tally(None, None, None, None) == -1


def test_struct_layouts_match_the_header(tmp_path):
    """The ctypes mirrors of the ABI structs have the C compiler's sizes and
    field offsets (gcc on include/hd_verify.h; no GPU)."""
    import shutil

    import pytest
    from hyperdrive_amd import _lib
    if not shutil.which("gcc"):
        pytest.skip("gcc absent")
    structs = {"hd_batch": _lib.HdBatch, "hd_batch_compact": _lib.HdBatchCompact, "hd_batch_out": _lib.HdBatchOut,
               "hd_tally_out": _lib.HdTallyOut, "hd_tally_ticket": _lib.HdTallyTicket}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "hd_verify.h"', "int main(void) {"]
    for cname, py in structs.items():
        lines.append(f'printf("{cname} size %zu\\n", sizeof({cname}));')
        for fname, _ in py._fields_:
            lines.append(f'printf("{cname} {fname} %zu\\n", offsetof({cname}, {fname}));')
    lines.append("return 0; }")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), "-o", str(exe), str(src)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split("\n")
    got = {}
    for line in out:
        if line:
            parts = line.split()
            got[(parts[0], parts[1])] = int(parts[2])
    for cname, py in structs.items():
        assert got[(cname, "size")] == ctypes.sizeof(py), cname
        for fname, _ in py._fields_:
            assert got[(cname, fname)] == getattr(py, fname).offset, (cname, fname)
