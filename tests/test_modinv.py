"""Bernstein-Yang divstep inversion (hyperdrive_amd/csrc/hd_modinv.h), host
build, against Python's pow(x, -1, m) for the group order n and the prime p,
on random values and on inputs with extreme bit patterns."""
import random

P = 2 ** 256 - 2 ** 32 - 977
N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141


def _inputs(m, rng, k):
    edge = [1, 2, 3, m - 1, m - 2, (m - 1) // 2, (m + 1) // 2, 2 ** 255 % m, 2 ** 128, 2 ** 128 - 1,
            (1 << 256) - 1 - (1 << 128), 0x5555555555555555555555555555555555555555555555555555555555555555 % m]
    edge += [(1 << k) % m for k in range(0, 256, 7)] + [(m - (1 << k)) % m for k in range(0, 256, 11)]
    return [e for e in edge if e] + [rng.randrange(1, m) for _ in range(k)]


def test_scalar_inverse(hostmath):
    rng = random.Random(31)
    for a in _inputs(N, rng, 3000):
        assert hostmath.sc("inv_divsteps", a) == pow(a, -1, N), hex(a)


def test_field_inverse(hostmath):
    rng = random.Random(32)
    for a in _inputs(P, rng, 3000):
        assert hostmath.fe("inv_divsteps", a)[0] == pow(a, -1, P), hex(a)
