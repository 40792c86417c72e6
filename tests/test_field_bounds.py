"""Limb bounds of the lazily reduced radix-2^29 field (hyperdrive_amd/csrc/hd_field.h).

Two layers:
* certification: the host build with -DHD_BOUNDS carries per-limb interval
  bounds through every operation and checks every precondition (64-bit
  column accumulators of fe_mul, 32-bit limbs of additions, K p >= subtrahend
  of fe_sub_k, tight outputs of the point formulas).  Running each formula
  once with operands at their class maxima certifies it for ALL inputs of
  those classes; the full recovery path is run on real messages as well.
* extremes: concrete worst-case limb values through mul / sqr / weak and full
  normalisation, checked against Python integers.
"""
import ctypes
import random

import numpy as np

P = 2 ** 256 - 2 ** 32 - 977
M29 = (1 << 29) - 1
M24 = (1 << 24) - 1
T = [M29, M29, M29 + (1 << 17)] + [M29] * 5 + [M24]


def val(limbs):
    return sum(int(x) << (29 * i) for i, x in enumerate(limbs))


def raw(hm, op, a, b=None):
    A = (ctypes.c_uint32 * 9)(*a)
    B = (ctypes.c_uint32 * 9)(*(b or [0] * 9))
    O = (ctypes.c_uint32 * 9)()
    hm.L.hdh_fe_raw(op, A, B, O)
    return list(O)


def failures(hm):
    buf = ctypes.create_string_buffer(256)
    n = hm.L.hdh_bound_failures(buf, 256)
    return n, buf.value.decode()


def is_tight(l):
    return all(x <= t for x, t in zip(l, T))


def b32(x):
    return x.to_bytes(32, "big")


def test_point_formulas_certified(oracle, hostmath_bounds):
    hm = hostmath_bounds
    hm.L.hdh_bound_certify.restype = ctypes.c_int
    rng = random.Random(5)
    for _ in range(4):
        Pp = oracle.point_mul(rng.randrange(1, oracle.N), oracle.G)
        Qq = oracle.point_mul(rng.randrange(1, oracle.N), oracle.G)
        n = hm.L.hdh_bound_certify(b32(Pp[0]), b32(Pp[1]), b32(Qq[0]), b32(Qq[1]))
        assert n == 0, failures(hm)


def test_recovery_path_within_bounds(oracle, hostmath_bounds):
    """every operation of recover() (sqrt, inversions, GLV ladder, affine
    conversion) on real signatures, with tracked bounds"""
    hm = hostmath_bounds
    for i in range(3):
        sk = oracle.signer_sk(i)
        d = oracle.sha256(bytes([i]))
        sig = oracle.sign(sk, d)
        v, pub = hm.recover(d, sig)
        assert v == 0
        assert failures(hm)[0] == 0, failures(hm)


def test_mul_bound_checker_rejects_overflow(hostmath_bounds):
    """the certifier is live: 3T x 3T may overflow a column and must be flagged"""
    hm = hostmath_bounds
    a = [3 * t for t in T]
    raw(hm, 0, a, a)
    n, what = failures(hm)
    assert n > 0 and "column" in what


def test_mul_sqr_worst_case_inputs(hostmath):
    rng = random.Random(21)
    cases = [(T, [7 * t for t in T]), ([2 * t for t in T], [3 * t for t in T]), (T, T)]
    cases += [([rng.randrange(2 * t + 1) for t in T], [rng.randrange(3 * t + 1) for t in T]) for _ in range(300)]
    for a, b in cases:
        r = raw(hostmath, 0, a, b)
        assert val(r) % P == val(a) * val(b) % P
        assert is_tight(r), r
        if all(x <= 2 * t for x, t in zip(a, T)):
            s = raw(hostmath, 1, a)
            assert val(s) % P == val(a) ** 2 % P
            assert is_tight(s), s


def test_weak_and_full_normalisation(hostmath):
    rng = random.Random(22)
    cases = [[0xFFFFFFF7] * 9, [0] * 9, T, [M29] * 8 + [M24]]
    for v in [P, P + 1, 2 ** 256 - 1, 2 ** 256 + 5, 2 ** 256 + 0x1000003D0, 2 * P - 1]:
        cases.append([(v >> (29 * i)) & M29 for i in range(8)] + [v >> 232])
    cases += [[rng.randrange(0xFFFFFFF8) for _ in range(9)] for _ in range(300)]
    for a in cases:
        w = raw(hostmath, 2, a)
        assert val(w) % P == val(a) % P
        assert is_tight(w), (a, w)
        n = raw(hostmath, 3, a)
        assert val(n) == val(a) % P
        assert all(x <= M29 for x in n[:8]) and n[8] <= M24


def test_point_ops_on_extreme_points(oracle, hostmath):
    """ecmult with points whose coordinates have long runs of 1-bits."""
    rng = random.Random(23)
    for _ in range(6):
        while True:
            x = (P - 1 - rng.randrange(1 << 20)) if rng.random() < 0.5 else (2 ** 255 - 1 - rng.randrange(1 << 20))
            R = oracle.lift_x(x % P, 1)
            if R is not None:
                break
        u1, u2 = rng.randrange(oracle.N), rng.randrange(oracle.N)
        want = oracle.point_add(oracle.point_mul(u1, oracle.G), oracle.point_mul(u2, R))
        assert hostmath.ecmult(R, u1, u2) == want
