"""Parity against the committed golden fixtures (tests/golden/, made by
tests/golden/make_golden.py).

CPU (-m "not gpu"): the oracle restatements (Python and C), the host build of
the device math headers, and OpenSSL reproduce every fixture.
GPU (-m gpu): the HIP path, called through the C ABI, reproduces every
fixture bit for bit -- verdicts, recovered signatories, valid bitmaps, the
first-wins tally and the quorum predicates -- with no oracle at run time.
"""
import glob
import json
import os

import numpy as np
import pytest

from util import OpenSSL, from_np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = sorted(os.path.basename(p)[len("verify_"):-len(".npz")] for p in glob.glob(os.path.join(GOLDEN, "verify_*.npz")))


def load_case(name):
    from hyperdrive_amd.verify import Batch
    z = np.load(os.path.join(GOLDEN, f"verify_{name}.npz"))  # allow_pickle=False (default)
    b = Batch(z["type"], z["height"], z["round"], z["valid_round"], z["value"], z["frm"], z["sig"])
    with open(os.path.join(GOLDEN, f"tally_{name}.json")) as fh:
        tj = json.load(fh)
    return b, z, tj


def tally_from_json(tj):
    count = {(h, r, t, bytes.fromhex(v)): c for h, r, t, v, c in tj["count"]}
    distinct = {(h, r, t): c for h, r, t, c in tj["distinct"]}
    distinct_any = {(h, r): c for h, r, c in tj["distinct_any"]}
    return count, distinct, distinct_any, tj["dup"]


def test_golden_cases_present():
    assert len(CASES) >= 7, CASES


def test_kats(oracle, coracle):
    with open(os.path.join(GOLDEN, "kats.json")) as fh:
        k = json.load(fh)
    for m, d in k["sha256"]:
        assert oracle.sha256(bytes.fromhex(m)).hex() == d
        assert coracle.sha256(bytes.fromhex(m)).hex() == d
    for e in k["ecrecover"]:
        v, pub = coracle.recover(bytes.fromhex(e["digest"]), bytes.fromhex(e["sig"]))
        assert v == 0 and pub.hex() == e["pub65"]
    for e in k["digests"]:
        value = bytes.fromhex(e["value"])
        assert oracle.message_digest(oracle.PREVOTE, e["h"], e["r"], e["vr"], value).hex() == e["vote"]
        assert coracle.digest(3, e["h"], e["r"], e["vr"], value).hex() == e["vote"]
        assert coracle.digest(1, e["h"], e["r"], e["vr"], value).hex() == e["propose"]


@pytest.mark.parametrize("name", CASES)
def test_c_oracle_and_host_headers_reproduce_fixture(coracle, hostmath, name):
    b, z, _ = load_case(name)
    compressed = int(z["compressed"])
    cv, crec = coracle.verify(b, z["admitted"], compressed, threads=4)
    assert cv.tolist() == z["verdict"].tolist()
    assert crec.tobytes() == z["recovered"].tobytes()
    adm_sorted = np.array(sorted(z["admitted"].tolist()), np.uint8)
    hv, hrec, _ = hostmath.verify(b, adm_sorted, compressed)
    assert hv.tolist() == z["verdict"].tolist()
    assert hrec.tobytes() == z["recovered"].tobytes()


@pytest.mark.parametrize("name", ["edges", "votes_100signers_tail"])
def test_python_oracle_reproduces_fixture(oracle, name):
    b, z, tj = load_case(name)
    ob = from_np(b)
    adm = [bytes(r) for r in z["admitted"]]
    vs, recs = oracle.verify_batch(ob, adm, int(z["compressed"]))
    assert vs == z["verdict"].tolist()
    assert b"".join(recs) == z["recovered"].tobytes()


@pytest.mark.parametrize("name", CASES)
def test_fixture_tally_and_openssl(oracle, name):
    b, z, tj = load_case(name)
    ob = from_np(b)
    t = oracle.tally(ob, z["verdict"].tolist())
    count, distinct, distinct_any, dup = tally_from_json(tj)
    assert t.count == count and t.distinct == distinct and t.distinct_any == distinct_any and t.dup == dup
    ossl = OpenSSL()
    for i in np.flatnonzero(z["verdict"] == 0)[:40]:
        d = oracle.message_digest(ob.mtype[i], ob.height[i], ob.round[i], ob.valid_round[i], ob.value[i])
        v, Q = oracle.recover(d, ob.sig[i])
        r, s = int.from_bytes(ob.sig[i][:32], "big"), int.from_bytes(ob.sig[i][32:64], "big")
        assert v == 0 and ossl.verify(d, r, s, oracle.pubkey_bytes(Q, False))


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_gpu_matches_golden(gpu, name):
    """Each fixture is verified twice on one context.  Pass 1 finds no known
    key, so every message takes the full recovery, which teaches the context
    the keys of the admitted signers it saw VALID.  Pass 2 then runs the
    known-key check (hd_fixedbase.h) on those signers' messages: its fallback
    count may not exceed the fixture's non-VALID messages plus the VALID ones
    of signers it could not have learned, and both passes must equal the
    golden verdicts, recovered signatories, bitmap, tally and decisions."""
    from hyperdrive_amd import quorum
    b, z, tj = load_case(name)
    v = gpu.Verifier(0, compressed=int(z["compressed"]))
    try:
        v.set_signatories(z["admitted"])
        for rnd in range(2):
            res, tal = v.process_batch(b)
            assert res.verdict.tolist() == z["verdict"].tolist(), rnd
            assert res.recovered.tobytes() == z["recovered"].tobytes(), rnd
            bits = np.unpackbits(res.valid_bitmap.view(np.uint8), bitorder="little")[: len(b)]
            assert bits.tolist() == (z["verdict"] == 0).astype(int).tolist()
            count, distinct, distinct_any, dup = tally_from_json(tj)
            assert tal.count == count
            assert tal.distinct == distinct
            assert tal.distinct_any == distinct_any
            assert tal.dup.tolist() == dup
            for d in tj["decisions"]:
                pv = bytes.fromhex(d["propose_value"]) if d["propose_value"] else None
                got = quorum.decide(tal, d["h"], d["r"], tj["f"], pv, pv is not None)
                assert got == d["decision"], d
            known, fallback = v.fastpath_stats()
            valid = z["verdict"] == 0
            if rnd == 0:
                # every VALID signer's key is learned from its first VALID message
                learned = len({b.frm[i].tobytes() for i in np.flatnonzero(valid)})
                assert known == learned
                assert fallback == len(b) - int((z["verdict"] == 7).sum())    # BAD_TYPE is decided up front
            else:
                # the known-key check decided every VALID message (a zero
                # window digit, ~2^-20 per message, would also fall back)
                assert fallback <= int((~valid).sum()), (fallback, int((~valid).sum()))
                if valid.any():
                    assert fallback < len(b)
    finally:
        v.close()


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_gpu_authenticate_golden(gpu, name):
    """hd_authenticate_batch_device on each fixture, after a verify pass has
    taught the context the keys: VALID and NOT_ADMITTED exactly the golden
    verdicts, every other message its golden verdict or NOT_AUTHENTIC (8),
    and NOT_AUTHENTIC only for Froms in the admitted set."""
    import torch
    from hyperdrive_amd.device import DeviceBatch, work_stream
    b, z, _ = load_case(name)
    if len(b) == 0:
        return
    v = gpu.Verifier(0, compressed=int(z["compressed"]))
    try:
        v.set_signatories(z["admitted"])
        v.verify_batch(b)
        db = DeviceBatch.from_host(b, "cuda")
        out = torch.full((len(b),), 255, dtype=torch.uint8, device="cuda")
        ws = work_stream()
        ws.wait_stream(torch.cuda.current_stream())
        v.authenticate_batch_device(db.c_struct(), out.data_ptr(), ws.cuda_stream)
        ws.synchronize()
        va, want = out.cpu().numpy(), z["verdict"]
        auth = np.isin(want, (0, 6))
        assert (va[auth] == want[auth]).all()
        assert not np.isin(va[~auth], (0, 6)).any()
        na = va == 8
        assert ((va == want) | na).all()
        adm = {bytes(x) for x in np.asarray(z["admitted"]).reshape(-1, 32)}
        assert all(b.frm[i].tobytes() in adm for i in np.flatnonzero(na))
    finally:
        v.close()


# Every kernel instantiation a context can select (include/hd_verify.h
# HD_VAR_*), one at a time from the defaults; the first entry is the default.
VARIANTS = [("default", None, None), ("verify_waves_2", "verify_waves", 2), ("verify_waves_4", "verify_waves", 4),
            ("sum_waves_2", "sum_waves", 2), ("sum_waves_3", "sum_waves", 3), ("sum_waves_4", "sum_waves", 4),
            ("sum_prefetch_2", "sum_prefetch", 2), ("split_k_8", "split_k", 8), ("split_k_16", "split_k", 16),
            ("recover_glv_g", "recover_g", 1), ("key_width_13", "key_width", 13), ("key_width_16", "key_width", 16),
            ("key_width_20", "key_width", 20), ("key_width_22", "key_width", 22),
            ("wave_prio_2", "wave_prio", 2), ("foreign_keys_0", "foreign_keys", 0), ("slow_lift_0", "slow_lift", 0)]


@pytest.mark.gpu
@pytest.mark.parametrize("label,key,value", VARIANTS, ids=[v[0] for v in VARIANTS])
def test_gpu_variants_match_golden(gpu, label, key, value):
    """Each selectable k_verify / k_fast_sums / known-key-check
    instantiation reproduces every golden fixture, through the full recovery
    (pass 1) and the known-key check (pass 2)."""
    for name in CASES:
        b, z, _ = load_case(name)
        v = gpu.Verifier(0, compressed=int(z["compressed"]))
        try:
            if key:
                v.set_variant(key, value)
            v.set_signatories(z["admitted"])
            # (foreign keys, on by default: pass 1 learns them, pass 2 builds
            # their tables, pass 3 checks with them)
            for rnd in range(2 if key == "foreign_keys" else 3):
                res = v.verify_batch(b)
                assert res.verdict.tolist() == z["verdict"].tolist(), (label, name, rnd)
                assert res.recovered.tobytes() == z["recovered"].tobytes(), (label, name, rnd)
        finally:
            v.close()


def test_variant_api_rejects_bad_values():
    import hyperdrive_amd._lib as L
    lib = L.load()
    assert lib.hd_ctx_set_variant(None, 0, 3) == L.HD_EINVAL
