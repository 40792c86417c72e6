"""The seeded synthetic workload (hd_gen.h) equals the oracle's definition of
it (oracle/hd_pyoracle.py gen_message) byte for byte, for every adversarial
class and both workload kinds."""
import numpy as np
import pytest


@pytest.mark.parametrize("kind,S,n,adv,start", [(0, 10, 150, 60, 0), (1, 7, 80, 40, 0), (0, 100, 40, 30, 123456),
                                                (1, 1000, 10, 0, 64 * 2001 - 3), (0, 4, 50, 100, 7)])
def test_generator_matches_oracle(oracle, hostmath, kind, S, n, adv, start):
    keys = oracle.KeyCache()
    ks = hostmath.keys(S)
    assert ks[0].tobytes() == b"".join(oracle.admitted_set(S, keys))
    assert ks[1].tobytes() == b"".join(keys.signatory(oracle.NONADMITTED_BASE + k) for k in range(16))
    hb, hcls = hostmath.gen(kind, start, n, S, adv, ks)
    ob, cls = oracle.gen_batch(kind, n, S, adv, start=start, keys=keys)
    assert hb.type.tolist() == ob.mtype
    assert hb.height.tolist() == ob.height and hb.round.tolist() == ob.round
    assert hb.valid_round.tolist() == ob.valid_round
    assert hb.value.tobytes() == b"".join(ob.value)
    assert hb.frm.tobytes() == b"".join(ob.frm)
    assert hb.sig.tobytes() == b"".join(ob.sig)
    assert hcls.tolist() == cls


def test_workload_shape(oracle):
    """C2 layout: signer = i % S, type = 2 + (i/S)%2, h = 1 + i/(2S), r = 0."""
    S = 100
    for i in [0, 1, 99, 100, 199, 200, 12345]:
        t, h, r, vr, v, signer = oracle.base_message(oracle.GEN_VOTES, i, S)
        assert signer == i % S and t == 2 + (i // S) % 2 and h == 1 + i // 200 and r == 0
    # C3: per round one propose from (h + r) % S then S prevotes then S precommits
    S = 1000
    per = 1 + 2 * S
    for r in [0, 1, 63]:
        t, h, rr, vr, v, signer = oracle.base_message(oracle.GEN_ROUNDS, r * per, S)
        assert t == oracle.PROPOSE and signer == (1 + r) % S and rr == r and vr == -1
        assert oracle.base_message(oracle.GEN_ROUNDS, r * per + 1, S)[0] == oracle.PREVOTE
        assert oracle.base_message(oracle.GEN_ROUNDS, r * per + S + 1, S)[0] == oracle.PRECOMMIT
