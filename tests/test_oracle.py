"""Pins the oracle before it is trusted.

The reference holds no byte-level golden vectors for this path, so the
restatement is pinned by: public known-answer tests (FIPS 180-2 SHA-256, the
secp256k1 generator, go-ethereum v1.9.5's published ecrecover vector from its
crypto tests), OpenSSL 3's independent ECDSA implementation, and the
reference's own property tests (sign -> Signatory(&hash) -> Equal,
process/message_test.go:145-158; hash determinism :133-143)."""
import hashlib
import os
import random
import struct

import numpy as np
import pytest

from util import OpenSSL, to_np


def test_sha256_kats(oracle, coracle):
    # FIPS 180-2 appendix B vectors
    assert oracle.sha256(b"abc").hex() == "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad"
    assert oracle.sha256(b"").hex() == "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855"
    m = b"abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq"
    assert oracle.sha256(m).hex() == "248d6a61d20638b8e5c026930c3e6039a33ce45964ff2167f6ecedd419db06c1"
    for n in range(0, 200):
        b = bytes((i * 7 + n) & 255 for i in range(n))
        assert coracle.sha256(b) == hashlib.sha256(b).digest()


def test_curve_constants(oracle):
    assert oracle.P % 4 == 3
    assert (oracle.GY ** 2 - oracle.GX ** 3 - 7) % oracle.P == 0
    assert oracle.point_mul(oracle.N, oracle.G) is None
    assert oracle.point_mul(1, oracle.G) == oracle.G


def test_go_ethereum_ecrecover_vector(oracle, coracle):
    # go-ethereum crypto tests (testmsg / testsig / testpubkey), pinned dependency v1.9.5
    msg = bytes.fromhex("ce0677bb30baa8cf067c88db9811f4333d131bf8bcf12fe7065d211dce971008")
    sig = bytes.fromhex("90f27b8b488db00b00606796d2987f6a5f59ae62ea05effe84fef5b8b0e54998"
                        "4a691139ad57a3f0b906637673aa2f63d1f55cb1a69199d4009eea23ceaddc9301")
    pub = bytes.fromhex("04e32df42865e97135acfb65f3bae71bdc86f4d49150ad6a440b6f15878109880a"
                        "0a2b2667f7e725ceea70c673093bf67663e0312623c8e091b13cf2c0f11ef652")
    v, Q = oracle.recover(msg, sig)
    assert v == oracle.VALID and oracle.pubkey_bytes(Q, False) == pub
    v2, pub2 = coracle.recover(msg, sig)
    assert v2 == 0 and pub2 == pub


def test_preimage_layout(oracle, coracle):
    """surge encoding: BE64 h || BE64 r [|| BE64 vr] || value; 48 / 56 bytes;
    NewPrevoteHash == NewPrecommitHash for the same (h, r, v) (message.go:172-186
    vs 270-284: no type tag)."""
    v = bytes(range(32))
    pre = oracle.vote_preimage(-1, 2 ** 63 - 1, v)
    assert len(pre) == 48 and pre[:8] == b"\xff" * 8 and pre[8:16] == b"\x7f" + b"\xff" * 7
    assert len(oracle.propose_preimage(1, 2, -1, v)) == 56
    for h, r, vr in [(0, 0, -1), (-1, -1, -1), (2 ** 63 - 1, 5, 3), (-2 ** 63, 0, 0)]:
        d2 = oracle.message_digest(oracle.PREVOTE, h, r, vr, v)
        d3 = oracle.message_digest(oracle.PRECOMMIT, h, r, vr, v)
        assert d2 == d3
        assert coracle.digest(2, h, r, vr, v) == d2 == coracle.digest(3, h, r, vr, v)
        assert coracle.digest(1, h, r, vr, v) == oracle.message_digest(oracle.PROPOSE, h, r, vr, v)


def test_sign_recover_roundtrip_and_openssl(oracle):
    """message_test.go:145-158: Sign -> Signatory(&hash) -> Equal, plus OpenSSL
    verification of every (digest, r, s) under the recovered key."""
    ossl = OpenSSL()
    rng = random.Random(7)
    for i in range(12):
        sk = oracle.signer_sk(i)
        assert ossl.pubkey(sk, False) == oracle.pubkey_bytes(oracle.pubkey_of(sk), False)
        assert ossl.pubkey(sk, True) == oracle.pubkey_bytes(oracle.pubkey_of(sk), True)
        h, r = rng.randrange(-2 ** 63, 2 ** 63), rng.randrange(-2 ** 63, 2 ** 63)
        d = oracle.message_digest(oracle.PREVOTE, h, r, -1, oracle.canonical_value(h, r))
        sig = oracle.sign(sk, d)
        rr, ss = int.from_bytes(sig[:32], "big"), int.from_bytes(sig[32:64], "big")
        assert ss <= oracle.N // 2 and sig[64] in (0, 1, 2, 3)
        v, Q = oracle.recover(d, sig)
        assert v == oracle.VALID and Q == oracle.pubkey_of(sk)
        assert ossl.verify(d, rr, ss, oracle.pubkey_bytes(Q, False))
        # high-S malleation recovers the same key (accepted by recover)
        mal = sig[:32] + (oracle.N - ss).to_bytes(32, "big") + bytes([sig[64] ^ 1])
        v2, Q2 = oracle.recover(d, mal)
        assert v2 == oracle.VALID and Q2 == Q


def test_rfc6979_nonce_known_structure(oracle):
    # determinism (message_test.go:133-143 analogue for signatures): same key+digest -> same sig
    sk = oracle.signer_sk(3)
    d = oracle.sha256(b"x")
    assert oracle.sign(sk, d) == oracle.sign(sk, d)
    assert oracle.sign(sk, d) != oracle.sign(oracle.signer_sk(4), d)


def test_adversarial_classes_produce_intended_verdicts(oracle):
    b, cls = oracle.gen_batch(oracle.GEN_VOTES, 260, 10, adv_pct=100)
    adm = oracle.admitted_set(10)
    vs, _ = oracle.verify_batch(b, adm)
    want = {1: {oracle.BAD_RECID}, 2: {oracle.BAD_RS}, 3: {oracle.BAD_RS}, 4: {oracle.NO_POINT},
            5: {oracle.NO_POINT}, 6: {oracle.NOT_ADMITTED}, 7: {oracle.SIGNATORY_MISMATCH},
            8: {oracle.VALID}, 9: {oracle.VALID}, 10: {oracle.INFINITY}, 11: {oracle.VALID}, 12: {oracle.VALID}}
    seen = set()
    for c, v in zip(cls, vs):
        seen.add(c)
        if c in want:
            assert v in want[c], (c, v)
        elif c == 0:
            assert v != oracle.VALID
    assert seen >= set(range(13))


@pytest.mark.parametrize("compressed", [True, False, 2, 3])
def test_c_oracle_matches_python_oracle(oracle, coracle, compressed):
    keys = oracle.KeyCache(compressed)
    for kind, n, S, adv in [(oracle.GEN_VOTES, 150, 10, 70), (oracle.GEN_ROUNDS, 60, 7, 40)]:
        ob, _ = oracle.gen_batch(kind, n, S, adv, keys=keys)
        adm = oracle.admitted_set(S, keys)
        vs, recs = oracle.verify_batch(ob, adm, compressed)
        nb = to_np(ob)
        cv, crec = coracle.verify(nb, np.frombuffer(b"".join(adm), np.uint8), compressed, threads=4)
        assert cv.tolist() == vs
        assert crec.tobytes() == b"".join(recs)


def test_oracle_openssl_on_all_valid_messages(oracle):
    ossl = OpenSSL()
    ob, cls = oracle.gen_batch(oracle.GEN_VOTES, 80, 10, adv_pct=50)
    for i in range(len(ob)):
        d = oracle.message_digest(ob.mtype[i], ob.height[i], ob.round[i], ob.valid_round[i], ob.value[i])
        v, Q = oracle.recover(d, ob.sig[i])
        if v == oracle.VALID:
            r = int.from_bytes(ob.sig[i][:32], "big")
            s = int.from_bytes(ob.sig[i][32:64], "big")
            assert ossl.verify(d, r, s, oracle.pubkey_bytes(Q, False)), i


def test_glv_port_baseline_equals_c_oracle(coracle, hostmath):
    """The 'port-glv' CPU baseline (oracle/glv_port.cpp, bench.py's
    cpu_baseline) gives the C oracle's verdicts and recovered signatories on
    the 30 % adversarial mix, on one and on several threads."""
    import subprocess
    from oracle_c import GlvPort
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    subprocess.run(["make", "-s", "-C", os.path.join(root, "oracle")], check=True)
    gp = GlvPort(os.path.join(root, "oracle", "_build", "libglvport.so"))
    sigs, foreign = hostmath.keys(50, True)
    b, _ = hostmath.gen(0, 3, 3000, 50, 30, (sigs, foreign))
    cv, crec = coracle.verify(b, sigs, True, threads=4)
    for th in (1, 5):
        v, rec = gp.verify(b, sigs, True, threads=th)
        assert v.tolist() == cv.tolist()
        assert rec.tobytes() == crec.tobytes()


def test_secp_class_port_equals_c_oracle(coracle, hostmath):
    """The 'port-secp-class' CPU baseline (oracle/secp_port.cpp: 5 x 52-bit
    field, GLV + wNAF Strauss ladder, divsteps inversions) gives the C
    oracle's verdicts and recovered signatories on the 30 % adversarial mix
    (every class: bad recid, r / s range, r + n >= p, no point, infinity,
    mismatch, not admitted, bad type), on one and on several threads, for the
    compressed and the uncompressed pubkey encodings."""
    import subprocess
    from oracle_c import SecpPort
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    subprocess.run(["make", "-s", "-C", os.path.join(root, "oracle")], check=True)
    sp = SecpPort(os.path.join(root, "oracle", "_build", "libsecpport.so"))
    for compressed in (True, False):
        sigs, foreign = hostmath.keys(50, compressed)
        b, _ = hostmath.gen(0, 3, 3000, 50, 30, (sigs, foreign))
        cv, crec = coracle.verify(b, sigs, compressed, threads=4)
        assert len(set(cv.tolist())) >= 7
        for th in (1, 5):
            v, rec = sp.verify(b, sigs, compressed, threads=th)
            assert v.tolist() == cv.tolist(), (compressed, th)
            assert rec.tobytes() == crec.tobytes(), (compressed, th)
