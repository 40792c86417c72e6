"""The device arithmetic (hyperdrive_amd/csrc/*.h), built for the host, checked
operation by operation against Python integers.  The kernels compile the same
source for gfx950; tests/test_gpu_*.py then check the GPU results end to end."""
import random

import pytest

from hostmath import b32


def _fe_inputs(oracle, rng, k=200):
    P = oracle.P
    edge = [0, 1, 2, 3, P - 1, P - 2, 2 ** 32, 2 ** 32 - 1, 2 ** 255, P - 2 ** 32, 0x1000003D1,
            2 ** 256 - 2 ** 32 - 978, 2 ** 224 - 1, (1 << 256) - 1 - (1 << 32) - 977 - 5]
    return [e % P for e in edge] + [rng.randrange(P) for _ in range(k)] + \
        [(P - rng.randrange(2 ** 40)) % P for _ in range(30)] + [rng.randrange(2 ** 40) for _ in range(30)]


def test_field_ops(oracle, hostmath):
    P = oracle.P
    rng = random.Random(11)
    vals = _fe_inputs(oracle, rng)
    for a in vals:
        b = rng.choice(vals)
        assert hostmath.fe("mul", a, b)[0] == a * b % P
        assert hostmath.fe("sqr", a)[0] == a * a % P
        assert hostmath.fe("add", a, b)[0] == (a + b) % P
        assert hostmath.fe("sub", a, b)[0] == (a - b) % P
        assert hostmath.fe("neg", a)[0] == (-a) % P


def test_field_inverse_and_sqrt_chains(oracle, hostmath):
    P = oracle.P
    rng = random.Random(12)
    for a in _fe_inputs(oracle, rng, 60):
        if a:
            assert hostmath.fe("inv", a)[0] == pow(a, P - 2, P)
        r, ok = hostmath.fe("sqrt", a)
        assert ok == (pow(a, (P - 1) // 2, P) in (0, 1))
        assert r == pow(a, (P + 1) // 4, P)


def test_scalar_ops(oracle, hostmath):
    N = oracle.N
    rng = random.Random(13)
    vals = [0, 1, 2, N - 1, N - 2, 2 ** 128, 2 ** 255, N // 2, N // 2 + 1] + [rng.randrange(N) for _ in range(200)]
    for a in vals:
        b = rng.choice(vals)
        assert hostmath.sc("mul", a, b) == a * b % N
        assert hostmath.sc("sqr", a) == a * a % N
        assert hostmath.sc("neg", a) == (-a) % N
    for a in vals[:60]:
        if a:
            assert hostmath.sc("inv", a) == pow(a, N - 2, N)
    for x in [0, N - 1, N, N + 5, 2 ** 256 - 1] + [rng.randrange(2 ** 256) for _ in range(100)]:
        assert hostmath.sc("reduce", x) == x % N


def test_booth_recoding(oracle, hostmath):
    rng = random.Random(14)
    for k in [0, 1, oracle.N - 1, 2 ** 255, 2 ** 256 - 1 - 2 ** 200] + [rng.randrange(oracle.N) for _ in range(100)]:
        for w, nw in ((4, 65), (8, 33)):
            ds = [hostmath.booth(k, w, j) for j in range(nw)]
            assert all(abs(d) <= 2 ** (w - 1) for d in ds)
            assert sum(d << (w * j) for j, d in enumerate(ds)) == k


def test_generator_table(oracle, hostmath):
    tab = hostmath.gtab()
    acc = None
    for k in range(128):
        acc = oracle.point_add(acc, oracle.G)
        assert tab[k] == acc


def test_ecmult(oracle, hostmath):
    rng = random.Random(15)
    R = oracle.point_mul(rng.randrange(1, oracle.N), oracle.G)
    cases = [(0, 0), (1, 0), (0, 1), (1, 1), (128, 8), (255, 9), (oracle.N - 1, 1), (1, oracle.N - 1)]
    cases += [(rng.randrange(oracle.N), rng.randrange(oracle.N)) for _ in range(15)]
    cases += [(rng.randrange(2 ** 16), rng.randrange(2 ** 16)) for _ in range(5)]
    for u1, u2 in cases:
        want = oracle.point_add(oracle.point_mul(u1, oracle.G), oracle.point_mul(u2, R))
        assert hostmath.ecmult(R, u1, u2) == want, (u1, u2)
    # R = G and R = -G: exercises the P == +-T branches of the addition law
    for RR in (oracle.G, oracle.point_neg(oracle.G)):
        for u1, u2 in [(1, 1), (5, oracle.N - 5), (2, 3), (rng.randrange(oracle.N), 7)]:
            want = oracle.point_add(oracle.point_mul(u1, oracle.G), oracle.point_mul(u2, RR))
            assert hostmath.ecmult(RR, u1, u2) == want, (u1, u2)


def test_signing_bit_exact(oracle, hostmath):
    for i in range(12):
        sk = oracle.signer_sk(i)
        assert hostmath.signer_sk(i) == sk
        d = oracle.sha256(bytes([i]) * (i + 1))
        assert hostmath.sign(sk, d) == oracle.sign(sk, d)


def test_recover_matches_oracle(oracle, hostmath):
    ob, _ = oracle.gen_batch(oracle.GEN_VOTES, 120, 10, adv_pct=80)
    for i in range(len(ob)):
        d = oracle.message_digest(ob.mtype[i], ob.height[i], ob.round[i], ob.valid_round[i], ob.value[i])
        v, Q = oracle.recover(d, ob.sig[i])
        hv, hQ = hostmath.recover(d, ob.sig[i])
        assert (hv, hQ) == (v, Q), i
