"""Per-kernel register use of a built library (CPU; reads the code objects' metadata).

    python scripts/kregs.py [lib.so] [name-filter]

Prints VGPRs (arch + acc, as allocated), SGPRs, scratch bytes and spill counts
per kernel, from the AMDHSA metadata note of each gfx950 code object in the
library's .hip_fatbin.  Waves per SIMD follow from the VGPR total (512 per lane)."""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"


def code_objects(lib, tmp):
    fat = os.path.join(tmp, "fatbin.bin")
    subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", lib, fat], check=True)
    data = open(fat, "rb").read()
    offs = [m.start() for m in re.finditer(re.escape(b"__CLANG_OFFLOAD_BUNDLE__"), data)] + [len(data)]
    out = []
    for k in range(len(offs) - 1):
        b = os.path.join(tmp, f"b{k}.bin")
        co = os.path.join(tmp, f"b{k}.co")
        open(b, "wb").write(data[offs[k]:offs[k + 1]])
        r = subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={b}", f"--output={co}"],
                           capture_output=True)
        if r.returncode == 0 and os.path.getsize(co):
            out.append(co)
    return out


def kernels(co):
    notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", co],
                           capture_output=True, text=True, check=True).stdout
    cur = {}
    for line in notes.splitlines():
        s = line.strip().lstrip("- ")
        if ":" not in s:
            continue
        k, _, v = s.partition(":")
        k, v = k.strip(), v.strip()
        if k == ".agpr_count":          # first key of a kernel's map
            if cur.get(".name"):
                yield cur
            cur = {}
        cur[k] = v
    if cur.get(".name"):
        yield cur


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "hyperdrive_amd", "_lib", "libhdverify.so")
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    with tempfile.TemporaryDirectory() as tmp:
        rows = []
        for co in code_objects(lib, tmp):
            for k in kernels(co):
                if filt in k[".name"]:
                    rows.append(k)
    for k in sorted(rows, key=lambda k: k[".name"]):
        v, a = int(k.get(".vgpr_count", 0)), int(k.get(".agpr_count", 0))
        tot = v + a if a == 0 else ((v + 3) // 4) * 4 + a
        print(f"{k['.name'][:60]:60s} vgpr {v:3d} agpr {a:3d} total {tot:3d} waves/SIMD {min(8, 512 // max(tot, 1))}"
              f" sgpr {k.get('.sgpr_count', '?'):>3s} scratch {k.get('.private_segment_fixed_size', '?'):>4s}"
              f" vspill {k.get('.vgpr_spill_count', '?')}")


if __name__ == "__main__":
    main()
