"""verify_msg (the per-lane body of k_verify), host-built, against the oracle
on adversarial batches -- both pubkey encodings, propose/vote mixes, BAD_TYPE,
duplicate and empty admitted sets."""
import numpy as np
import pytest

from util import from_np, to_np


@pytest.mark.parametrize("compressed", [True, False, 2])
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
