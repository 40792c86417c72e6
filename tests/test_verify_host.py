"""verify_msg (the per-lane body of k_verify), host-built, against the oracle
on adversarial batches -- both pubkey encodings, propose/vote mixes, BAD_TYPE,
duplicate and empty admitted sets."""
import numpy as np
import pytest

from util import from_np, to_np


@pytest.mark.parametrize("compressed", [True, False, 2, 3])
@pytest.mark.parametrize("kind,S,n,adv", [(0, 10, 140, 70), (1, 7, 70, 50)])
def test_verify_matches_oracle(oracle, hostmath, compressed, kind, S, n, adv):
    keys = oracle.KeyCache(compressed)
    ob, _ = oracle.gen_batch(kind, n, S, adv, keys=keys)
    adm = sorted(oracle.admitted_set(S, keys))
    vs, recs = oracle.verify_batch(ob, adm, compressed)
    nb = to_np(ob)
    ver, rec, sgn = hostmath.verify(nb, np.frombuffer(b"".join(adm), np.uint8), compressed)
    assert ver.tolist() == vs
    assert rec.tobytes() == b"".join(recs)
    for i in range(n):
        if vs[i] == oracle.VALID:
            assert adm[sgn[i]] == ob.frm[i]
        else:
            assert sgn[i] == -1


def test_bad_type_and_empty_admitted(oracle, hostmath):
    ob, _ = oracle.gen_batch(oracle.GEN_VOTES, 20, 4, 0)
    nb = to_np(ob)
    nb.type[3] = 0
    nb.type[4] = 4      # Timeout (not a signed message)
    nb.type[5] = 255
    ver, _, _ = hostmath.verify(nb, np.zeros((0, 32), np.uint8))
    assert ver[3] == ver[4] == ver[5] == oracle.BAD_TYPE
    others = [int(v) for i, v in enumerate(ver) if i not in (3, 4, 5)]
    assert set(others) == {oracle.NOT_ADMITTED}
    adm = sorted(oracle.admitted_set(4))
    ver2, _, _ = hostmath.verify(nb, np.frombuffer(b"".join(adm[:1]), np.uint8))
    ref, _ = oracle.verify_batch(from_np(nb), adm[:1])
    assert ver2.tolist() == ref


def test_pubkey_hash_all_encodings(oracle, hostmath):
    """sha256_pubkey of hd_sha256.h (host build of the device header) against
    the oracle's id.NewSignatory encodings, for coordinates of every byte length
    0..32 -- including X.Bytes() || Y.Bytes() preimages short enough for one
    SHA-256 block (55 bytes or less), which no on-curve key reaches in practice."""
    import random
    rng = random.Random(0x57121)
    pairs = []
    for lx in range(33):
        for ly in (0, 1, 9, 23, 24, 31, 32, rng.randrange(33)):
            x = rng.getrandbits(8 * lx) | (1 << (8 * lx - 1)) if lx else 0
            y = rng.getrandbits(8 * ly) | (1 << (8 * ly - 1)) if ly else 0
            pairs.append((x, y))
    for x, y in pairs:
        for fmt in (0, 1, 2, 3):
            want = oracle.sha256(oracle.pubkey_bytes((x, y), fmt))
            assert hostmath.pubkey_hash(fmt, x, y) == want, (fmt, hex(x), hex(y))
    # the one-block branch really is exercised
    assert any(len(oracle.pubkey_bytes(p, 3)) <= 55 for p in pairs)
