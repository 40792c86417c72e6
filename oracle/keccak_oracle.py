"""Keccak-f[1600] sponge restated from FIPS 202 (SURVEY §8(f)4 digest lane).

TEST INFRASTRUCTURE ONLY: the checker of hd_keccak.h / include/hd_digest.h
in tests/; the product never imports it.

The reference never calls Keccak; this lane is pinned by
  * FIPS 202 itself: round constants from the rc(t) LFSR (Algorithm 5),
    rotation offsets from (t+1)(t+2)/2 along the (x, y) -> (y, 2x+3y) walk
    (Algorithm 2), both derived here rather than tabulated;
  * hashlib.sha3_256 (the same permutation with pad byte 0x06) on many inputs;
  * public Keccak-256 known answers: "" -> c5d24601...5d85a470,
    "abc" -> 4e03657a...2d6c45 (tests/test_keccak.py).
"""
from __future__ import annotations

import struct

MASK = (1 << 64) - 1
RATE = 136                      # bytes, capacity 512 -> 256-bit output


def _rc_bit(t: int) -> int:
    """rc(t) of FIPS 202 Algorithm 5 (LFSR x^8 + x^6 + x^5 + x^4 + 1)."""
    if t % 255 == 0:
        return 1
    r = [1, 0, 0, 0, 0, 0, 0, 0]
    for _ in range(t % 255):
        r = [0] + r
        r[0] ^= r[8]
        r[4] ^= r[8]
        r[5] ^= r[8]
        r[6] ^= r[8]
        r = r[:8]
    return r[0]


ROUND_CONSTANTS = []
for ir in range(24):
    rc = 0
    for j in range(7):
        rc |= _rc_bit(j + 7 * ir) << ((1 << j) - 1)
    ROUND_CONSTANTS.append(rc)

RHO = [[0] * 5 for _ in range(5)]     # RHO[x][y]
_x, _y = 1, 0
for _t in range(24):
    RHO[_x][_y] = ((_t + 1) * (_t + 2) // 2) % 64
    _x, _y = _y, (2 * _x + 3 * _y) % 5


def _rot(v: int, n: int) -> int:
    return ((v << n) | (v >> (64 - n))) & MASK if n else v


def keccak_f1600(a):
    """a: list of 25 lanes, index x + 5y."""
    for ir in range(24):
        c = [a[x] ^ a[x + 5] ^ a[x + 10] ^ a[x + 15] ^ a[x + 20] for x in range(5)]
        d = [c[(x - 1) % 5] ^ _rot(c[(x + 1) % 5], 1) for x in range(5)]
        a = [a[i] ^ d[i % 5] for i in range(25)]
        b = [0] * 25
        for x in range(5):
            for y in range(5):
                b[y + 5 * ((2 * x + 3 * y) % 5)] = _rot(a[x + 5 * y], RHO[x][y])
        a = [b[x + 5 * y] ^ ((~b[(x + 1) % 5 + 5 * y]) & b[(x + 2) % 5 + 5 * y]) for y in range(5) for x in range(5)]
        a[0] ^= ROUND_CONSTANTS[ir]
    return a


def sponge256(data: bytes, pad: int) -> bytes:
    """256-bit output, rate 136 B; pad = 0x01 (Keccak-256) or 0x06 (SHA3-256)."""
    m = bytearray(data)
    m.append(pad)
    while len(m) % RATE:
        m.append(0)
    m[-1] |= 0x80
    a = [0] * 25
    for off in range(0, len(m), RATE):
        lanes = struct.unpack_from("<17Q", m, off)
        for k in range(17):
            a[k] ^= lanes[k]
        a = keccak_f1600(a)
    return struct.pack("<4Q", *a[:4])


def keccak256(data: bytes) -> bytes:
    return sponge256(data, 0x01)


def sha3_256(data: bytes) -> bytes:
    return sponge256(data, 0x06)


PAD = {1: 0x01, 2: 0x06}     # HD_DIGEST_KECCAK256, HD_DIGEST_SHA3_256


def preimage(mtype: int, h: int, r: int, vr: int, value: bytes) -> bytes:
    """surge preimage (process/message.go:53-78 Propose, 165-186 / 263-284 votes)."""
    if mtype == 1:
        return struct.pack(">qqq", h, r, vr) + value
    return struct.pack(">qq", h, r) + value
