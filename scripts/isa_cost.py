#!/usr/bin/env python3
"""Static VALU cost of a kernel's loop bodies from its gfx950 assembly.

Weights are the measured issue costs of scripts/valu_probe.hip on MI355X
(cycles per wave-instruction per SIMD at 8 waves/SIMD): plain 32-bit VOP1/VOP2
ALU ops ~2.25, VOP3-only and 64-bit ops (v_mad_u64_u32, v_lshrrev_b64,
v_lshl_add_u64, v_add3_u32, v_alignbit_b32, v_bfe_u32, ...) ~4.3.

Usage: python scripts/isa_cost.py file.s [kernel-substring]
Prints, per kernel, the largest loop-body blocks with instruction counts and
weighted cycles.
"""
import re
import sys
from collections import Counter

FAST = {"v_add_u32_e32", "v_sub_u32_e32", "v_subrev_u32_e32", "v_and_b32_e32", "v_or_b32_e32", "v_xor_b32_e32",
        "v_lshrrev_b32_e32", "v_lshlrev_b32_e32", "v_ashrrev_i32_e32", "v_mov_b32_e32", "v_not_b32_e32",
        "v_cndmask_b32_e32", "v_max_u32_e32", "v_min_u32_e32", "v_max_i32_e32", "v_min_i32_e32"}


def cost(op):
    if op.startswith("s_") or op.startswith("scratch_") or op.startswith("ds_") or op.startswith("global_") \
            or op.startswith("buffer_"):
        return 0.0
    if op in FAST:
        return 2.25
    if op.startswith("v_"):
        return 4.3
    return 0.0


def blocks(lines):
    name, body = None, []
    for ln in lines:
        m = re.match(r"^(\.LBB\w+|_\w+):", ln)
        if m:
            if name:
                yield name, body
            name, body = m.group(1), []
            continue
        t = ln.strip()
        if t and not t.startswith(";") and not t.startswith("."):
            body.append(t.split()[0])
    if name:
        yield name, body


def main():
    path = sys.argv[1]
    want = sys.argv[2] if len(sys.argv) > 2 else None
    src = open(path).read().splitlines()
    # split by kernel
    kern, cur = {}, None
    for ln in src:
        m = re.match(r"^(_Z\w+):", ln)
        if m:
            cur = m.group(1)
            kern[cur] = []
        if cur:
            kern[cur].append(ln)
            if "s_endpgm" in ln:
                cur = None
    for k, lines in kern.items():
        if want and want not in k:
            continue
        tot = Counter()
        print(f"== {k}")
        rows = []
        for name, body in blocks(lines):
            c = Counter(body)
            tot.update(c)
            w = sum(cost(op) * n for op, n in c.items())
            rows.append((w, name, len(body), c["v_mad_u64_u32"]))
        for w, name, n, m in sorted(rows, reverse=True)[:6]:
            print(f"  {name:14s} {n:6d} instr  {m:4d} mad_u64  {w:9.0f} cyc")
        w = sum(cost(op) * n for op, n in tot.items())
        print(f"  total {sum(tot.values())} instr, weighted {w:.0f} cyc; top: {tot.most_common(12)}")


if __name__ == "__main__":
    main()
