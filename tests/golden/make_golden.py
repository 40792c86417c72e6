#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/ (test data only).

The reference (Go, tuanggolt/hyperdrive) cannot run in this container and its
own tests hold no byte-level vectors for this path, so the
fixtures are produced by the CPU restatement (oracle/hd_pyoracle.py), after it
is pinned by:
  * FIPS 180-2 SHA-256 known answers,
  * go-ethereum v1.9.5's published ecrecover vector (crypto tests: testmsg /
    testsig / testpubkey), recorded in kats.json,
  * OpenSSL 3's independent ECDSA verifier: every VALID message's
    (digest, r, s) verifies under the recovered key (checked here, at
    generation time, and again in tests/test_golden.py).

Files (all deterministic; re-running this script reproduces them byte for byte):
  kats.json               SHA-256 KATs, the go-ethereum vector, preimage digests
                          at the int64 extremes (process/message.go:53-78,
                          165-186, 263-284; surge BE64).
  verify_<case>.npz       an SoA batch (hd_batch layout) + admitted set +
                          expected verdicts and recovered signatories.
  tally_<case>.json       expected first-wins logs/counts (process.go:823-892)
                          and the quorum predicates for a few (h, r).

Usage: python tests/golden/make_golden.py [case ...]   (about a minute, pure Python;
       naming cases regenerates only those)
"""
from __future__ import annotations

import hashlib
import json
import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)

import hd_pyoracle as O  # noqa: E402

# (name, generator kind, n, signatories, adversarial %, start, pubkey format:
#  True = SEC1 compressed, False = SEC1 uncompressed, 2 = raw X || Y,
#  3 = X.Bytes() || Y.Bytes())
CASES = [
    ("votes_allclasses", O.GEN_VOTES, 260, 10, 100, 0, True),
    ("votes_mix30", O.GEN_VOTES, 200, 10, 30, 0, True),
    ("rounds_mix40", O.GEN_ROUNDS, 150, 7, 40, 0, True),
    ("votes_uncompressed", O.GEN_VOTES, 120, 10, 60, 0, False),
    ("votes_raw64", O.GEN_VOTES, 120, 10, 60, 0, O.PUBKEY_RAW64),
    ("votes_100signers_tail", O.GEN_VOTES, 64, 100, 30, 999_936, True),
]

INT64_EDGES = [0, 1, -1, 2 ** 63 - 1, -2 ** 63, 2 ** 32, -(2 ** 31)]

# Signer indices whose public keys have a leading zero byte in Y (58, 504) or
# X (560, 570), so X.Bytes() || Y.Bytes() is 63 bytes, not 64; 691 (Y) signs
# from outside the admitted set.
STRIP_ADMITTED = [58, 504, 560, 570, 0, 1, 2, 3]
STRIP_FOREIGN = 691


def kats():
    out = {"sha256": [
        ["", hashlib.sha256(b"").hexdigest()],
        ["616263", "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad"],
        [b"abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq".hex(),
         "248d6a61d20638b8e5c026930c3e6039a33ce45964ff2167f6ecedd419db06c1"],
    ]}
    for m, d in out["sha256"]:
        assert O.sha256(bytes.fromhex(m)).hex() == d
    # go-ethereum v1.9.5 crypto/crypto_test.go: testmsg, testsig, testpubkey
    out["ecrecover"] = [{
        "digest": "ce0677bb30baa8cf067c88db9811f4333d131bf8bcf12fe7065d211dce971008",
        "sig": "90f27b8b488db00b00606796d2987f6a5f59ae62ea05effe84fef5b8b0e54998"
               "4a691139ad57a3f0b906637673aa2f63d1f55cb1a69199d4009eea23ceaddc9301",
        "pub65": "04e32df42865e97135acfb65f3bae71bdc86f4d49150ad6a440b6f15878109880a"
                 "0a2b2667f7e725ceea70c673093bf67663e0312623c8e091b13cf2c0f11ef652",
    }]
    v, Q = O.recover(bytes.fromhex(out["ecrecover"][0]["digest"]), bytes.fromhex(out["ecrecover"][0]["sig"]))
    assert v == O.VALID and O.pubkey_bytes(Q, False).hex() == out["ecrecover"][0]["pub65"]
    rng = random.Random(0x48595045)
    digests = []
    for h in INT64_EDGES:
        for r in INT64_EDGES[:5]:
            value = bytes(rng.randrange(256) for _ in range(32)) if rng.random() < 0.7 else O.NIL_VALUE
            vr = rng.choice([-1, 0, 5, 2 ** 63 - 1])
            digests.append({"h": h, "r": r, "vr": vr, "value": value.hex(),
                            "vote": O.message_digest(O.PREVOTE, h, r, vr, value).hex(),
                            "propose": O.message_digest(O.PROPOSE, h, r, vr, value).hex()})
    out["digests"] = digests
    return out


def edge_batch(keys, S):
    """Honest votes/proposes at the int64 extremes of (h, r, vr), NilValue,
    and messages of every invalid type tag (BAD_TYPE)."""
    b = O.Batch()
    rng = random.Random(0x5EED)
    i = 0
    for h in INT64_EDGES:
        for r in (0, -1, 2 ** 63 - 1):
            for t in (O.PROPOSE, O.PREVOTE, O.PRECOMMIT):
                j = i % S
                vr = rng.choice([-1, 0, 2 ** 63 - 1, -2 ** 63])
                value = O.NIL_VALUE if i % 5 == 0 else bytes(rng.randrange(256) for _ in range(32))
                d = O.message_digest(t, h, r, vr, value)
                b.append(t, h, r, vr, value, keys.signatory(j), O.sign(keys.sk(j), d))
                i += 1
    for t in (0, 4, 5, 255):
        value = bytes(32)
        d = O.message_digest(O.PREVOTE, 1, 0, -1, value)
        b.append(t, 1, 0, -1, value, keys.signatory(0), O.sign(keys.sk(0), d))
    return b


def stripped_batch(keys):
    """Votes and proposes of the STRIP_ADMITTED signers (honest, double votes,
    signatures under another signer's From, a corrupted s, a non-admitted
    signer whose key also has a short coordinate)."""
    b = O.Batch()
    rng = random.Random(0x5742)
    for r in range(3):
        for t in (O.PROPOSE, O.PREVOTE, O.PRECOMMIT):
            for j in STRIP_ADMITTED:
                value = O.canonical_value(5, r) if rng.random() < 0.8 else bytes(rng.randrange(256) for _ in range(32))
                vr = -1 if t != O.PROPOSE else r - 1
                d = O.message_digest(t, 5, r, vr, value)
                b.append(t, 5, r, vr, value, keys.signatory(j), O.sign(keys.sk(j), d))
    for i, j in enumerate(STRIP_ADMITTED):
        value = bytes([i + 1]) * 32
        d = O.message_digest(O.PREVOTE, 5, 1, -1, value)
        b.append(O.PREVOTE, 5, 1, -1, value, keys.signatory(j), O.sign(keys.sk(j), d))        # double vote
        other = STRIP_ADMITTED[(i + 1) % len(STRIP_ADMITTED)]
        b.append(O.PRECOMMIT, 5, 2, -1, value, keys.signatory(other),
                 O.sign(keys.sk(j), O.message_digest(O.PRECOMMIT, 5, 2, -1, value)))        # From of another
        d = O.message_digest(O.PRECOMMIT, 5, 0, -1, value)
        sig = bytearray(O.sign(keys.sk(j), d))
        sig[40] ^= 0x10
        b.append(O.PRECOMMIT, 5, 0, -1, value, keys.signatory(j), bytes(sig))                # corrupted s
        d = O.message_digest(O.PREVOTE, 5, r, -1, value)
        b.append(O.PREVOTE, 5, r, -1, value, keys.signatory(STRIP_FOREIGN), O.sign(keys.sk(STRIP_FOREIGN), d))
    return b


def batch_arrays(ob):
    n = len(ob)
    return dict(
        type=np.array(ob.mtype, np.uint8), height=np.array(ob.height, np.int64),
        round=np.array(ob.round, np.int64), valid_round=np.array(ob.valid_round, np.int64),
        value=np.frombuffer(b"".join(ob.value), np.uint8).reshape(n, 32),
        frm=np.frombuffer(b"".join(ob.frm), np.uint8).reshape(n, 32),
        sig=np.frombuffer(b"".join(ob.sig), np.uint8).reshape(n, 65))


def openssl_check(ob, verdicts):
    from util import OpenSSL
    ossl = OpenSSL()
    for i in range(len(ob)):
        if verdicts[i] != O.VALID:
            continue
        d = O.message_digest(ob.mtype[i], ob.height[i], ob.round[i], ob.valid_round[i], ob.value[i])
        v, Q = O.recover(d, ob.sig[i])
        r = int.from_bytes(ob.sig[i][:32], "big")
        s = int.from_bytes(ob.sig[i][32:64], "big")
        assert v == O.VALID and ossl.verify(d, r, s, O.pubkey_bytes(Q, False)), i


def tally_json(ob, verdicts, S):
    t = O.tally(ob, verdicts)
    f = O.thresholds(S)[0]
    dec = []
    for (h, r) in sorted(t.distinct_any)[:12]:
        for pv in (None, O.canonical_value(h, r)):
            dec.append({"h": h, "r": r, "propose_value": pv.hex() if pv else None,
                        "decision": O.decide_round(t, h, r, f, pv, pv is not None)})
    return {
        "signatories": S, "f": f,
        "count": sorted([[h, r, ty, v.hex(), c] for (h, r, ty, v), c in t.count.items()]),
        "distinct": sorted([[h, r, ty, c] for (h, r, ty), c in t.distinct.items()]),
        "distinct_any": sorted([[h, r, c] for (h, r), c in t.distinct_any.items()]),
        "dup": t.dup,
        "decisions": dec,
    }


def main():
    if not sys.argv[1:]:
        with open(os.path.join(HERE, "kats.json"), "w") as fh:
            json.dump(kats(), fh, indent=1, sort_keys=True)
    cases = list(CASES) + [("edges", None, 0, 10, 0, 0, True),
                           ("votes_xystripped", "strip", 0, len(STRIP_ADMITTED), 0, 0, O.PUBKEY_XY_STRIPPED)]
    only = sys.argv[1:]
    for name, kind, n, S, adv, start, compressed in cases:
        if only and name not in only:
            continue
        keys = O.KeyCache(compressed)
        if kind is None:
            ob, cls = edge_batch(keys, S), []
        elif kind == "strip":
            ob, cls = stripped_batch(keys), []
        else:
            ob, cls = O.gen_batch(kind, n, S, adv, start=start, keys=keys)
        adm = ([keys.signatory(j) for j in STRIP_ADMITTED] if kind == "strip" else O.admitted_set(S, keys))
        verdicts, recs = O.verify_batch(ob, adm, compressed)
        openssl_check(ob, verdicts)
        arrs = batch_arrays(ob)
        np.savez_compressed(
            os.path.join(HERE, f"verify_{name}.npz"), **arrs,
            admitted=np.frombuffer(b"".join(adm), np.uint8).reshape(S, 32),
            compressed=np.array(int(compressed), np.uint8),
            verdict=np.array(verdicts, np.uint8),
            recovered=np.frombuffer(b"".join(recs), np.uint8).reshape(len(ob), 32),
            adv_class=np.array(cls, np.int8))
        with open(os.path.join(HERE, f"tally_{name}.json"), "w") as fh:
            json.dump(tally_json(ob, verdicts, S), fh, indent=0, sort_keys=True)
        print(f"{name}: {len(ob)} messages, verdicts {np.bincount(verdicts, minlength=8).tolist()}")


if __name__ == "__main__":
    main()
