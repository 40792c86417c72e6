"""Worst-case limb bounds of the lazily reduced radix-2^26 field
(hyperdrive_amd/csrc/hd_field.h): multiplier inputs up to L (limbs < 2^30, top
< 2^25.5), weak normalisation of anything < 2^32, and the T output bound."""
import ctypes
import random

import numpy as np

P = 2 ** 256 - 2 ** 32 - 977
M26 = (1 << 26) - 1
T_LIMB = (1 << 26) + (1 << 24)
T_TOP = (1 << 22) + 1


def val(limbs):
    return sum(int(x) << (26 * i) for i, x in enumerate(limbs))


def raw(hostmath, op, a, b=None):
    f = hostmath.L.hdh_fe_raw
    A = (ctypes.c_uint32 * 10)(*a)
    B = (ctypes.c_uint32 * 10)(*(b or [0] * 10))
    O = (ctypes.c_uint32 * 10)()
    f(op, A, B, O)
    return list(O)


def _limbs(rng, lo_max, top_max, extreme=False):
    if extreme:
        return [lo_max - 1] * 9 + [top_max - 1]
    return [rng.randrange(lo_max) for _ in range(9)] + [rng.randrange(top_max)]


def is_tight(l):
    return all(x < T_LIMB for x in l[:9]) and l[9] < T_TOP


L_TOP = int(2 ** 25.5)   # top-limb bound of a multiplier input (largest producer: 2r < 2^25.33)


def test_mul_sqr_worst_case_inputs(hostmath):
    rng = random.Random(21)
    cases = [(_limbs(rng, 1 << 30, L_TOP, True), _limbs(rng, 1 << 30, L_TOP, True))]
    cases += [(_limbs(rng, 1 << 30, L_TOP), _limbs(rng, 1 << 30, L_TOP)) for _ in range(300)]
    cases += [([M26] * 9 + [(1 << 22) - 1], [M26] * 9 + [(1 << 22) - 1])]
    for a, b in cases:
        r = raw(hostmath, 0, a, b)
        assert val(r) % P == val(a) * val(b) % P
        assert is_tight(r), r
        s = raw(hostmath, 1, a)
        assert val(s) % P == val(a) ** 2 % P
        assert is_tight(s), s


def test_weak_and_full_normalisation(hostmath):
    rng = random.Random(22)
    cases = [[(1 << 32) - (1 << 6) - 1] * 9 + [(1 << 31) - 1], [0] * 10, [M26] * 9 + [(1 << 22) - 1]]
    # values in [p, 2^256) and just above 2^256
    for v in [P, P + 1, 2 ** 256 - 1, 2 ** 256 + 5, 2 ** 256 + 0x1000003D0]:
        cases.append([(v >> (26 * i)) & M26 for i in range(9)] + [v >> 234])
    cases += [[rng.randrange((1 << 32) - (1 << 6)) for _ in range(9)] + [rng.randrange(1 << 31)] for _ in range(300)]
    for a in cases:
        w = raw(hostmath, 2, a)
        assert val(w) % P == val(a) % P
        assert is_tight(w), (a, w)
        n = raw(hostmath, 3, a)
        assert val(n) == val(a) % P
        assert all(x <= M26 for x in n[:9]) and n[9] < (1 << 22)


def test_point_ops_on_extreme_points(oracle, hostmath):
    """ecmult with points whose coordinates have long runs of 1-bits."""
    rng = random.Random(23)
    for _ in range(6):
        # pick x with many ones, lift to a point
        while True:
            x = (P - 1 - rng.randrange(1 << 20)) if rng.random() < 0.5 else (2 ** 255 - 1 - rng.randrange(1 << 20))
            R = oracle.lift_x(x % P, 1)
            if R is not None:
                break
        u1, u2 = rng.randrange(oracle.N), rng.randrange(oracle.N)
        want = oracle.point_add(oracle.point_mul(u1, oracle.G), oracle.point_mul(u2, R))
        assert hostmath.ecmult(R, u1, u2) == want
