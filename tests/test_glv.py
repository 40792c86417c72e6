"""GLV endomorphism: constants, the scalar split, and the 4-scalar ladder
(hyperdrive_amd/csrc/hd_group.h ecmult_glv), host build vs the oracle."""
import math
import random

LAM = 0x5363AD4CC05C30E0A5261C028812645A122E22EA20816678DF02967C1B23BD72
BETA = 0x7AE96A2B657C07106E64479EAC3434E99CF0497512F58995C1396C28719501EE


def test_endomorphism_constants(oracle):
    N, P = oracle.N, oracle.P
    assert pow(LAM, 3, N) == 1 and LAM != 1
    assert pow(BETA, 3, P) == 1 and BETA != 1
    assert oracle.point_mul(LAM, oracle.G) == (BETA * oracle.GX % P, oracle.GY)
    # lattice basis (a1, b1), (a2, b2) from the extended Euclid on (n, lambda)
    a1, b1 = 0x3086D221A7D46BCDE86C90E49284EB15, -0xE4437ED6010E88286F547FA90ABFE4C3
    a2, b2 = 0x114CA50F7A8E2F3F657C1108D9D44CFD8, 0x3086D221A7D46BCDE86C90E49284EB15
    assert (a1 + b1 * LAM) % N == 0 and (a2 + b2 * LAM) % N == 0
    assert a1 * b2 - a2 * b1 == N
    assert max(abs(a1), abs(b1), abs(a2), abs(b2)) < 2 ** 129


def test_lambda_table(oracle, hostmath):
    tab = hostmath.gtab()
    for k in range(128):
        assert tab[128 + k] == oracle.point_mul(LAM, tab[k])


def test_split(oracle, hostmath):
    N = oracle.N
    rng = random.Random(41)
    ks = [0, 1, 2, N - 1, N // 2, N // 2 + 1, LAM, N - LAM, 2 ** 128, 2 ** 255] + [rng.randrange(N) for _ in range(3000)]
    for k in ks:
        k1, k2 = hostmath.split(k)
        assert (k1 + k2 * LAM) % N == k
        for x in (k1, k2):
            mag = N - x if x > N // 2 else x
            assert mag < 2 ** 128, hex(k)


def test_ecmult_glv(oracle, hostmath):
    rng = random.Random(42)
    for _ in range(12):
        R = oracle.point_mul(rng.randrange(1, oracle.N), oracle.G)
        u1, u2 = rng.randrange(oracle.N), rng.randrange(oracle.N)
        want = oracle.point_add(oracle.point_mul(u1, oracle.G), oracle.point_mul(u2, R))
        assert hostmath.ecmult_glv(R, u1, u2) == want
    # degenerate: R = +-G, lambda G; zero scalars; cancellation to infinity
    G = oracle.G
    LG = oracle.point_mul(LAM, G)
    for R, u1, u2 in [(G, 1, 1), (G, 5, oracle.N - 5), (oracle.point_neg(G), 3, 3), (LG, LAM, 1),
                      (LG, 0, 7), (G, 0, 0), (G, 7, 0), (LG, oracle.N - LAM, 1)]:
        want = oracle.point_add(oracle.point_mul(u1, G), oracle.point_mul(u2, R))
        assert hostmath.ecmult_glv(R, u1, u2) == want, (u1, u2)


def test_ecmult_glv_fixed_base_g(oracle, hostmath):
    """ecmult_glv_fbg: u2 R by the GLV ladder, u1 G by fixed-base additions
    from a G table in an accumulator of its own, joined by one exact Jacobian
    addition -- the same point as ecmult_glv / the oracle, including zero
    scalars, the join cancelling (u1 G = -u2 R: infinity) and the join
    doubling (u1 G = u2 R)."""
    N, G = oracle.N, oracle.G
    rng = random.Random(43)
    cases = []
    for _ in range(10):
        k = rng.randrange(1, N)
        cases.append((k, rng.randrange(N), rng.randrange(N)))
    for k in (1, 2, 7, N - 1, LAM):
        u2 = rng.randrange(1, N)
        cases += [(k, (-u2 * k) % N, u2), (k, u2 * k % N, u2), (k, 0, u2), (k, rng.randrange(N), 0), (k, 0, 0),
                  (k, 1, 0), (k, N - 1, 1), (k, 2 ** 255 % N, 3)]
    for k, u1, u2 in cases:
        R = oracle.point_mul(k, G)
        want = oracle.point_add(oracle.point_mul(u1, G), oracle.point_mul(u2, R))
        got = hostmath.ecmult_glv_fbg8(R, u1, u2)
        assert got == want, (hex(k), hex(u1), hex(u2))
        assert got == hostmath.ecmult_glv(R, u1, u2)
