"""GPU parity: k_verify (through the C ABI) against the oracle, and the GPU
generator against the oracle's workload definition."""
import numpy as np
import pytest

from util import from_np, to_np

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def verifier(gpu):
    v = gpu.Verifier(0)
    yield v
    v.close()


@pytest.mark.parametrize("compressed", [True, False, 2, 3])
@pytest.mark.parametrize("kind,S,n,adv", [(0, 10, 300, 60), (1, 7, 150, 40), (0, 100, 257, 30), (1, 1000, 2001 + 5, 10)])
def test_verify_parity_vs_oracle(gpu, oracle, kind, S, n, adv, compressed):
    v = gpu.Verifier(0, compressed=compressed)
    keys = oracle.KeyCache(compressed)
    ob, _ = oracle.gen_batch(kind, min(n, 400), S, adv, keys=keys) if S < 1000 else _rounds_head(oracle, keys, n)
    adm = oracle.admitted_set(S, keys)
    v.set_signatories(adm)
    res = v.verify_batch(to_np(ob))
    vs, recs = oracle.verify_batch(ob, adm, compressed)
    assert res.verdict.tolist() == vs
    assert res.recovered.tobytes() == b"".join(recs)
    bits = np.unpackbits(res.valid_bitmap.view(np.uint8), bitorder="little")[: len(ob)]
    assert bits.tolist() == [int(x == oracle.VALID) for x in vs]
    v.close()


def _rounds_head(oracle, keys, n):
    # C3 shape (1000 signers) without signing 2001 messages in Python: the
    # first 40 messages of round 0 plus a few from round 1
    b1, c1 = oracle.gen_batch(oracle.GEN_ROUNDS, 40, 1000, 10, keys=keys)
    b2, c2 = oracle.gen_batch(oracle.GEN_ROUNDS, 5, 1000, 10, start=2001, keys=keys)
    for i in range(len(b2)):
        b1.append(b2.mtype[i], b2.height[i], b2.round[i], b2.valid_round[i], b2.value[i], b2.frm[i], b2.sig[i])
    return b1, c1 + c2


@pytest.mark.parametrize("kind,S,n,adv,start", [(0, 10, 300, 60, 0), (1, 7, 150, 40, 0), (0, 100, 64, 30, 999_936)])
def test_gpu_generator_matches_oracle(verifier, oracle, kind, S, n, adv, start):
    from hyperdrive_amd.device import generate
    keys = oracle.KeyCache()
    ks = verifier.gen_keys(S)
    assert ks[0].tobytes() == b"".join(oracle.admitted_set(S, keys))
    db, _, _ = generate(verifier, kind, n, S, adv, start=start, keys=ks)
    hb = db.to_host()
    ob, cls = oracle.gen_batch(kind, n, S, adv, start=start, keys=keys)
    assert hb.type.tolist() == ob.mtype
    assert hb.height.tolist() == ob.height and hb.round.tolist() == ob.round
    assert hb.value.tobytes() == b"".join(ob.value)
    assert hb.frm.tobytes() == b"".join(ob.frm)
    assert hb.sig.tobytes() == b"".join(ob.sig)
    assert db.adv_class.cpu().numpy().tolist() == cls


def test_edge_cases(verifier, oracle):
    keys = oracle.KeyCache()
    adm = oracle.admitted_set(4, keys)
    verifier.set_signatories(adm + adm[:2])          # duplicates in the admitted set are harmless
    empty = to_np(oracle.Batch())
    res = verifier.verify_batch(empty)
    assert len(res.verdict) == 0
    for n in (1, 31, 33, 63, 64, 65, 127):             # ragged sizes around the 32/64 bitmap words
        ob, _ = oracle.gen_batch(oracle.GEN_VOTES, n, 4, 40, keys=keys)
        res = verifier.verify_batch(to_np(ob))
        vs, _ = oracle.verify_batch(ob, adm)
        assert res.verdict.tolist() == vs
        bits = np.unpackbits(res.valid_bitmap.view(np.uint8), bitorder="little")[:n]
        assert bits.tolist() == [int(x == 0) for x in vs]
    ob, _ = oracle.gen_batch(oracle.GEN_VOTES, 20, 4, 0, keys=keys)
    nb = to_np(ob)
    nb.type[[2, 3, 4]] = [0, 4, 200]
    nb.valid_round = None                              # optional field
    res = verifier.verify_batch(nb)
    ref, _ = oracle.verify_batch(from_np(nb), adm)
    assert res.verdict.tolist() == ref
    assert res.verdict[2] == res.verdict[3] == res.verdict[4] == oracle.BAD_TYPE
    verifier.set_signatories([])                       # empty admitted set: nothing is admitted
    res = verifier.verify_batch(to_np(ob))
    assert set(res.verdict.tolist()) == {oracle.NOT_ADMITTED}


def test_full_size_c2_properties(verifier, oracle, coracle):
    """1M messages (BASELINE configs[1]): every honest message must verify to its
    own signer (by construction), the bitmap must agree with the verdicts, and a
    seeded sample must match the C oracle bit for bit."""
    import torch
    from hyperdrive_amd.device import generate
    N, S = 1 << 20, 100
    ks = verifier.gen_keys(S)
    verifier.set_signatories(ks[0])
    db, _, _ = generate(verifier, 0, N, S, 0, keys=ks)
    verdict = torch.empty(N, dtype=torch.uint8, device="cuda")
    signer = torch.empty(N, dtype=torch.int32, device="cuda")
    rec = torch.empty((N, 32), dtype=torch.uint8, device="cuda")
    bm = torch.empty(N // 32, dtype=torch.int32, device="cuda")
    from hyperdrive_amd.device import work_stream
    stream = work_stream().cuda_stream
    verifier.verify_batch_device(db.c_struct(), verdict.data_ptr(), rec.data_ptr(), signer.data_ptr(), bm.data_ptr(),
                                 stream)
    torch.cuda.synchronize()
    assert int((verdict != 0).sum()) == 0
    idx = torch.arange(N, device="cuda", dtype=torch.int64)
    assert bool((signer.long() == idx % S).all())
    assert bool((rec == db.frm).all())
    assert int(bm.view(torch.uint8).cpu().numpy().astype(np.uint8).sum()) == 255 * (N // 8)
    # sample vs the C oracle
    rng = np.random.default_rng(5)
    pick = np.sort(rng.choice(N, 512, replace=False))
    hb = db.to_host()
    from hyperdrive_amd.verify import Batch
    sb = Batch(hb.type[pick], hb.height[pick], hb.round[pick], hb.valid_round[pick], hb.value[pick], hb.frm[pick],
               hb.sig[pick])
    cv, crec = coracle.verify(sb, ks[0], True, threads=8)
    assert cv.tolist() == verdict.cpu().numpy()[pick].tolist()
    assert crec.tobytes() == rec.cpu().numpy()[pick].tobytes()


@pytest.mark.parametrize("variants", [{}, {"split_k": 16}], ids=["default", "k16"])
def test_adversarial_full_mix_vs_c_oracle(gpu, oracle, coracle, variants):
    """C5-style mix: 30 % adversarial across all classes, 64k messages, checked
    message by message against the C oracle on a context of its own: pass 1
    (no key known: the full recovery) teaches it the 100 keys, pass 2 runs the
    known-key check for the honest messages (its fallback list is only the
    adversarial share); both passes equal the oracle.  Also at 16 messages
    per inversion (the default takes 8 below 2^20 - 2^16 messages, 16 above)."""
    from hyperdrive_amd.device import generate
    N, S = 65536, 100
    v = gpu.Verifier(0)
    try:
        for k, x in variants.items():
            v.set_variant(k, x)
        ks = v.gen_keys(S)
        v.set_signatories(ks[0])
        db, _, _ = generate(v, 0, N, S, 30, keys=ks)
        hb = db.to_host()
        cv, crec = coracle.verify(hb, ks[0], True, threads=16)
        for rnd in range(2):
            res = v.verify_batch(hb)
            assert res.verdict.tolist() == cv.tolist(), rnd
            assert res.recovered.tobytes() == crec.tobytes(), rnd
            known, fallback = v.fastpath_stats()
            if rnd == 0:
                assert known == S and fallback == N
            else:
                assert fallback <= int((cv != 0).sum()) + 5     # + rare zero window digits
        hist = np.bincount(res.verdict, minlength=8)
        assert hist[0] > 0.7 * N and all(hist[k] > 0 for k in range(1, 7))
    finally:
        v.close()


def test_authenticate_vs_c_oracle(gpu, coracle):
    """hd_authenticate_batch_device (the replica ingress's call) on the 30 %
    adversarial mix: before the keys are known every verdict is the oracle's
    (full recovery); once they are, VALID and NOT_ADMITTED are still exactly
    the oracle's, every other message is the oracle's verdict or
    NOT_AUTHENTIC, NOT_AUTHENTIC only where From is admitted, and the
    fallback list shrinks to what the known-key check cannot decide (Froms
    outside the admitted set, the early verdicts' lift checks).  A full
    verify on the same context afterwards is unaffected."""
    import torch
    from hyperdrive_amd.device import DeviceBatch, generate, work_stream
    N, S = 65536, 100
    v = gpu.Verifier(0)
    try:
        ks = v.gen_keys(S)
        v.set_signatories(ks[0])
        db, _, _ = generate(v, 0, N, S, 30, keys=ks)
        hb = db.to_host()
        cv, crec = coracle.verify(hb, ks[0], True, threads=16)
        admitted = {x.tobytes() for x in ks[0]}
        from_adm = np.array([hb.frm[i].tobytes() in admitted for i in range(N)])
        ws = work_stream()
        out = torch.empty(N, dtype=torch.uint8, device="cuda")
        fallbacks = []
        for rnd in range(3):
            out.fill_(255)
            v.authenticate_batch_device(db.c_struct(), out.data_ptr(), ws.cuda_stream)
            ws.synchronize()
            va = out.cpu().numpy()
            fallbacks.append(v.fastpath_stats()[1])
            if rnd == 0:
                assert va.tolist() == cv.tolist()          # no key known yet: the full recovery
                continue
            auth = np.isin(cv, (0, 6))
            assert (va[auth] == cv[auth]).all()
            assert not np.isin(va[~auth], (0, 6)).any()
            na = va == 8
            assert ((va == cv) | na).all()
            assert na.sum() > 0.05 * N and from_adm[na].all()
        assert fallbacks[2] < 0.5 * int((cv != 0).sum())
        res = v.verify_batch(hb)
        assert res.verdict.tolist() == cv.tolist()
        assert res.recovered.tobytes() == crec.tobytes()
    finally:
        v.close()


def test_foreign_keys_vs_c_oracle(gpu, coracle):
    """HD_VAR_FOREIGN_KEYS: the 30 % adversarial mix's authenticated senders
    outside the admitted set (16 foreign keys) are learned from their
    NOT_ADMITTED recoveries; once their tables are built their messages take
    the known-key check.  Every pass equals the C oracle (verdicts and
    recovered signatories, NOT_ADMITTED included), the fallback list shrinks by
    the foreign share, and authenticate_batch_device then needs no full
    recovery for them either."""
    import torch
    from hyperdrive_amd.device import generate, work_stream
    N, S = 65536, 100
    v = gpu.Verifier(0)
    try:
        v.set_variant("foreign_keys", 16)
        ks = v.gen_keys(S)
        v.set_signatories(ks[0])
        db, _, _ = generate(v, 0, N, S, 30, keys=ks)
        hb = db.to_host()
        cv, crec = coracle.verify(hb, ks[0], True, threads=16)
        fallback = []
        for rnd in range(4):
            res = v.verify_batch(hb)
            assert res.verdict.tolist() == cv.tolist(), rnd
            assert res.recovered.tobytes() == crec.tobytes(), rnd
            bits = np.unpackbits(res.valid_bitmap.view(np.uint8), bitorder="little")[:N]
            assert bits.tolist() == (cv == 0).astype(int).tolist()
            fallback.append(v.fastpath_stats()[1])
        n_foreign = int((cv == 6).sum())
        assert n_foreign > 1000
        # the same batch on a context without foreign keys: its steady fallback
        # includes every NOT_ADMITTED message, this one's none of them
        # (foreign keys are on by default: turned off here before the set, so
        # the baseline does not depend on the environment)
        v0 = gpu.Verifier(0)
        try:
            v0.set_variant("foreign_keys", 0)
            v0.set_signatories(ks[0])
            for _ in range(3):
                v0.verify_batch(hb)
            base = v0.fastpath_stats()[1]
        finally:
            v0.close()
        assert base >= n_foreign, (base, n_foreign)
        assert all(f <= base - n_foreign + 5 for f in fallback[1:]), (fallback, base, n_foreign)
        # turning the variant off at the next set change stops the foreign
        # check (the reserved block stays, unused): every NOT_ADMITTED message
        # takes the full recovery again, with the same outputs
        v.set_variant("foreign_keys", 0)
        v.set_signatories(ks[0])
        for _ in range(3):
            res = v.verify_batch(hb)
            assert res.verdict.tolist() == cv.tolist()
            assert res.recovered.tobytes() == crec.tobytes()
        assert v.fastpath_stats()[1] >= n_foreign
        v.set_variant("foreign_keys", 16)
        v.set_signatories(ks[0])
        for _ in range(3):   # learn the foreign keys again, build, check
            res = v.verify_batch(hb)
            assert res.verdict.tolist() == cv.tolist()
        assert v.fastpath_stats()[1] <= base - n_foreign + 5
        ws = work_stream()
        out = torch.empty(N, dtype=torch.uint8, device="cuda")
        v.authenticate_batch_device(db.c_struct(), out.data_ptr(), ws.cuda_stream)
        ws.synchronize()
        va = out.cpu().numpy()
        auth = np.isin(cv, (0, 6))
        assert (va[auth] == cv[auth]).all() and not np.isin(va[~auth], (0, 6)).any()
        assert v.fastpath_stats()[1] <= 5          # nothing left for the full recovery
    finally:
        v.close()


def _subset(hb, idx):
    from hyperdrive_amd.verify import Batch
    return Batch(hb.type[idx], hb.height[idx], hb.round[idx],
                 None if hb.valid_round is None else hb.valid_round[idx], hb.value[idx], hb.frm[idx], hb.sig[idx])


def test_foreign_slot_eviction(gpu, coracle):
    """Foreign-key slots are not first come, first served for good: with 4
    slots, 4 throwaway Froms (one NOT_ADMITTED message each) claim them first;
    a fifth foreign sender with many messages then counts recoveries while it
    has no slot, and a later call hands it the slot of the coldest throwaway
    key (hd_fastverify.hip fb_evict), after which its messages take the
    known-key check.  Every call's verdicts and recovered signatories equal
    the C oracle; the throwaway keys' messages stay exact after losing their
    slots."""
    from hyperdrive_amd.device import generate
    N, S = 65536, 100
    v = gpu.Verifier(0)
    try:
        v.set_variant("foreign_keys", 4)
        ks = v.gen_keys(S)
        v.set_signatories(ks[0])
        db, _, _ = generate(v, 0, N, S, 30, keys=ks)
        hb = db.to_host()
        cv, _ = coracle.verify(hb, ks[0], True, threads=16)
        na = np.flatnonzero(cv == 6)                       # NOT_ADMITTED: authenticated foreign senders
        froms = {}
        for i in na.tolist():
            froms.setdefault(hb.frm[i].tobytes(), []).append(i)
        senders = sorted(froms.values(), key=len, reverse=True)
        assert len(senders) >= 5 and len(senders[0]) >= 50, [len(x) for x in senders]
        hot = senders[0]
        junk = [x[0] for x in senders[1:5]]
        valid = np.flatnonzero(cv == 0)[:4096].tolist()
        first = _subset(hb, np.array(junk + valid))
        fv, frec = coracle.verify(first, ks[0], True, threads=16)
        for _ in range(3):                                 # the junk keys claim and build the 4 slots
            r = v.verify_batch(first)
            assert r.verdict.tolist() == fv.tolist() and r.recovered.tobytes() == frec.tobytes()
        assert v.foreign_stats() == (4, 0)
        second = _subset(hb, np.array(hot + valid))
        sv, srec = coracle.verify(second, ks[0], True, threads=16)
        falls = []
        for _ in range(6):
            r = v.verify_batch(second)
            assert r.verdict.tolist() == sv.tolist() and r.recovered.tobytes() == srec.tobytes()
            falls.append(v.fastpath_stats()[1])
        ready, evicted = v.foreign_stats()
        assert evicted == 1 and ready == 4, (ready, evicted, falls)
        assert falls[0] >= len(hot) and falls[-1] == 0, falls   # the hot sender reached the known-key check
        for _ in range(2):                                 # the evicted key's message: exact, via the recovery
            r = v.verify_batch(first)
            assert r.verdict.tolist() == fv.tolist() and r.recovered.tobytes() == frec.tobytes()
    finally:
        v.close()


def test_fallback_burst_after_clean_batches(gpu, coracle):
    """The fallback kernels (k_slow_lift, k_verify over the leftover list) size
    their grids by the latest list length seen (hd_fastverify.hip
    fallback_blocks).  After honest batches (no leftovers: the smallest grid)
    a 30 %-adversarial batch on the same context has ~10k leftovers that the
    small grids walk grid-stride; every verdict and signatory must still
    equal the C oracle, and the next adversarial batch too (grids sized by
    the burst)."""
    from hyperdrive_amd.device import generate
    N, S = 65536, 100
    v = gpu.Verifier(0)
    try:
        ks = v.gen_keys(S)
        v.set_signatories(ks[0])
        clean, _, _ = generate(v, 0, N, S, 0, keys=ks)
        hc = clean.to_host()
        for _ in range(3):                          # learn the keys, then two calls with no leftovers
            v.verify_batch(hc)
        assert v.fastpath_stats()[1] == 0
        adv, _, _ = generate(v, 0, N, S, 30, keys=ks, start=N)
        ha = adv.to_host()
        cv, crec = coracle.verify(ha, ks[0], True, threads=16)
        for rnd in range(2):
            res = v.verify_batch(ha)
            assert res.verdict.tolist() == cv.tolist(), rnd
            assert res.recovered.tobytes() == crec.tobytes(), rnd
        assert v.fastpath_stats()[1] > 1000
    finally:
        v.close()


def test_c4_16m_sharded_emulation(verifier, coracle):
    """BASELINE configs[3] (16M messages, sharded over 8 GPUs) on one GPU: the
    8 rank shards (shard_range) verified one after another into their bitmap
    slices give exactly the single-launch bitmap; all 16M honest votes are
    VALID with signer = i mod S; a seeded sample matches the C oracle; the
    tally from the concatenated shard bitmaps equals the tally from the
    single-launch verdicts."""
    import torch
    from hyperdrive_amd.device import generate, work_stream
    from hyperdrive_amd.shard import shard_range
    from hyperdrive_amd._lib import HdBatch
    N, S, W = 1 << 24, 100, 8
    ks = verifier.gen_keys(S)
    verifier.set_signatories(ks[0])
    db, _, _ = generate(verifier, 0, N, S, 0, keys=ks)
    ws = work_stream()
    verdict = torch.empty(N, dtype=torch.uint8, device="cuda")
    signer = torch.empty(N, dtype=torch.int32, device="cuda")
    bm_full = torch.zeros(N // 32, dtype=torch.int32, device="cuda")
    verifier.verify_batch_device(db.c_struct(), verdict.data_ptr(), None, signer.data_ptr(), bm_full.data_ptr(),
                                 ws.cuda_stream)
    bm_sh = torch.zeros(N // 32, dtype=torch.int32, device="cuda")
    v_sh = torch.empty(N, dtype=torch.uint8, device="cuda")
    for k in range(W):
        lo, hi = shard_range(N, k, W)
        sh = HdBatch(hi - lo, db.type.data_ptr() + lo, db.height.data_ptr() + 8 * lo, db.round.data_ptr() + 8 * lo,
                     db.valid_round.data_ptr() + 8 * lo, db.value.data_ptr() + 32 * lo,
                     db.frm.data_ptr() + 32 * lo, db.sig.data_ptr() + 65 * lo)
        verifier.verify_batch_device(sh, v_sh.data_ptr() + lo, None, None, bm_sh.data_ptr() + 4 * (lo // 32),
                                     ws.cuda_stream)
    ws.synchronize()
    assert torch.equal(bm_full, bm_sh) and torch.equal(verdict, v_sh)
    assert int((verdict != 0).sum()) == 0
    idx = torch.arange(N, device="cuda", dtype=torch.int64)
    assert bool((signer.long() == idx % S).all())
    rng = np.random.default_rng(16)
    pick = np.sort(rng.choice(N, 256, replace=False))
    p = torch.from_numpy(pick).cuda()
    from hyperdrive_amd.verify import Batch
    sb = Batch(db.type[p].cpu().numpy(), db.height[p].cpu().numpy(), db.round[p].cpu().numpy(),
               db.valid_round[p].cpu().numpy(), db.value[p].cpu().numpy(), db.frm[p].cpu().numpy(),
               db.sig[p].cpu().numpy())
    cv, _ = coracle.verify(sb, ks[0], True, threads=8)
    assert cv.tolist() == [0] * len(pick)
    # tally: bitmap path (what every rank runs after the all-gather) == verdict path
    import ctypes
    from hyperdrive_amd import _lib
    lib = _lib.load()
    t1, a1 = verifier._tally_struct(N)
    t2, a2 = verifier._tally_struct(N)
    full = db.c_struct()
    assert lib.hd_tally_device_bitmap(verifier.handle, ctypes.byref(full), bm_sh.data_ptr(), ctypes.byref(t1),
                                      ws.cuda_stream) == 0
    assert lib.hd_tally_device(verifier.handle, ctypes.byref(full), verdict.data_ptr(), ctypes.byref(t2),
                               ws.cuda_stream) == 0
    assert (t1.n_hr, t1.n_counts) == (t2.n_hr, t2.n_counts)
    for k in ("count_height", "count_round", "count_type", "count_n", "hr_height", "hr_prevotes", "hr_precommits",
              "hr_any"):
        m = t1.n_counts if k.startswith("count") else t1.n_hr
        assert np.array_equal(a1[k][:m], a2[k][:m]), k
    assert t1.n_hr == N // (2 * S) + (1 if N % (2 * S) else 0)


@pytest.mark.timeout(900)
def test_c4_16m_adversarial_bit_exact(gpu):
    """BASELINE configs[3] at full size with the C5 mix: 16,777,216 messages
    from the C4 generator (100 signatories) with 30 % adversarial messages
    across all 13 classes (duplicates and double votes included).  Every
    verdict and recovered signatory of the product path (two passes on a
    fresh context: the cold full recovery that learns the keys, then the
    known-key check) equals the host restatement (oracle/secp_port.cpp,
    bit-exact with the C oracle), and the library's tally of the GPU verdicts
    equals the C oracle's tally of the host verdicts row for row, with every
    round's quorum decisions (quorum.decide vs oracle_tally's predicate bits;
    process/process.go:574-582, 696-702; message_test.go:145-158)."""
    import time

    import torch
    import bitexact
    from hyperdrive_amd.device import generate, work_stream
    N, S = 1 << 24, 100
    v = gpu.Verifier(0)
    try:
        ks = v.gen_keys(S)
        v.set_signatories(ks[0])
        db, _, _ = generate(v, 0, N, S, 30, keys=ks)
        ws = work_stream()
        verdict = torch.empty(N, dtype=torch.uint8, device="cuda")
        rec = torch.empty((N, 32), dtype=torch.uint8, device="cuda")
        bm = torch.zeros(N // 32, dtype=torch.int32, device="cuda")
        outs = []
        for _ in range(2):
            t0 = time.perf_counter()
            v.verify_batch_device(db.c_struct(), verdict.data_ptr(), rec.data_ptr(), None, bm.data_ptr(),
                                  ws.cuda_stream)
            ws.synchronize()
            outs.append((verdict.cpu().numpy(), rec.cpu().numpy(), time.perf_counter() - t0))
        (v0, r0, cold_s), (v1, r1, warm_s) = outs
        assert v.fastpath_stats()[0] >= S                    # the second pass ran the known-key check
        hb = db.to_host()
        res = bitexact.full_check(v, hb, v1, r1, ks[0])
        print("c4 16M adversarial:", {**res, "gpu_cold_s": cold_s, "gpu_warm_s": warm_s})
        assert np.array_equal(v0, v1) and np.array_equal(r0, r1)
        assert res["verdicts"] and res["signatories"], res
        assert res["tally_rows"] and res["decisions"], res
        hist = res["verdict_hist"]
        assert hist[0] > N // 2 and sum(1 for c in hist[1:] if c) >= 5, hist   # the classes are there
        assert res["commits"] > 0
        bits = np.unpackbits(bm.cpu().numpy().view(np.uint8), bitorder="little")[:N]
        assert np.array_equal(bits, (v1 == 0).astype(np.uint8))
    finally:
        v.close()


def _zero_digit_rows(oracle, S):
    """Signatures whose known-key check scalars u1 = m / s and u2 = r / s have
    zero window digits (in the 24-bit G windows and the 16- and 20-bit key
    windows), made by choosing u1, u2 first: k = u1 + u2 d, R = k G, r = R.x,
    s = r / u2, m = u1 s (the digest is supplied, hd_verify_batch_digest_device).
    Zero digits otherwise come up ~2^-W per window; here every message has
    several, including a sum that starts late (u1's low windows zero, or u1 = 0)."""
    import random
    O = oracle
    keys = O.KeyCache()
    rng = random.Random(5)
    ones = lambda lo, hi: ((1 << (hi - lo + 1)) - 1) << lo
    pairs = [
        (2 ** 100 + 2 ** 30 + 5, 2 ** 200 + 7),                   # sparse: most digits zero, any width
        (0, rng.randrange(1, O.N)),                              # u1 = 0: the sum starts in the key windows
        (rng.randrange(1, 2 ** 200) << 24, rng.randrange(1, O.N)),  # G window 0 zero: starts at window 1
        (rng.randrange(1, 2 ** 180) << 48, rng.randrange(1, O.N)),  # G windows 0, 1 zero
        (rng.randrange(1, O.N) | ones(71, 95), rng.randrange(1, O.N)),   # G window 3 all ones (Booth zero)
        (rng.randrange(1, O.N), rng.randrange(1, 2 ** 239)),     # key top window zero (20-bit tables)
        (rng.randrange(1, O.N), rng.randrange(1, O.N) | ones(99, 119)),  # 20-bit key window 5 all ones
        (rng.randrange(1, O.N), rng.randrange(1, O.N) & ~ones(63, 79)),  # 16-bit key window 4 zero
        (rng.randrange(1, O.N), rng.randrange(1, O.N) & ~ones(51, 65)),  # 13-bit key window 4 zero
        (rng.randrange(1, O.N), rng.randrange(1, 2 ** 246)),     # key top window zero (13-bit tables)
        (rng.randrange(1, O.N), rng.randrange(1, 2 ** 241)),     # key top window zero (22-bit tables)
        (rng.randrange(1, O.N), rng.randrange(1, O.N) & ~ones(87, 109)),  # 22-bit key window 4 zero
        (rng.randrange(1, O.N), 2 ** 128 + 1),                   # sparse u2
        (rng.randrange(1, O.N), rng.randrange(1, O.N)),          # control
    ]
    rows, digests = [], []
    for j, (u1, u2) in enumerate(pairs):
        for signer, claimed in ((j % S, j % S), (j % S, (j + 1) % S)):   # honest, then a mismatching From
            d = keys.sk(signer)
            k = (u1 + u2 * d) % O.N
            R = O.point_mul(k, O.G)
            r = R[0] % O.N
            v = (R[1] & 1) | (2 if R[0] >= O.N else 0)
            s = r * pow(u2, -1, O.N) % O.N
            m = u1 * s % O.N
            sig = r.to_bytes(32, "big") + s.to_bytes(32, "big") + bytes([v])
            val = bytes(rng.randrange(256) for _ in range(32))
            rows.append((O.PREVOTE, 1 + j, 0, -1, val, keys.signatory(claimed), sig))
            digests.append(m.to_bytes(32, "big"))
    return rows, digests, keys


@pytest.mark.parametrize("key_width", [13, 16, 20, 22])
def test_zero_window_digits_vs_oracle(gpu, oracle, key_width):
    """The known-key check's rare branch (k_fast_sums: a wavefront with a
    zero window digit adds the window's entry 0 and takes it off again; a sum
    that has not started starts at the first non-zero window) on messages
    built to have zero digits: verdicts and recovered signatories equal the
    oracle's recovery through the full recovery (pass 1) and the known-key
    check (passes 2, 3), where only the mismatching Froms fall back."""
    import torch
    from hyperdrive_amd.device import DeviceBatch, work_stream
    from hyperdrive_amd.digest import verify_digest_device
    from hyperdrive_amd.verify import Batch
    O = oracle
    S = 4
    rows, digests, keys = _zero_digit_rows(O, S)
    want, wrec = [], []
    for (t, h, r, vr, val, frm, sig), dg in zip(rows, digests):
        verdict, Q = O.recover(dg, sig)
        if verdict == O.VALID:
            got = O.signatory_of_pub(Q, True)
            verdict = O.VALID if got == frm else O.SIGNATORY_MISMATCH
            wrec.append(got)
        else:
            wrec.append(bytes(32))
        want.append(verdict)
    assert want.count(O.VALID) == len(rows) // 2
    v = gpu.Verifier(0)
    try:
        v.set_variant("key_width", key_width)
        v.set_signatories(np.frombuffer(b"".join(keys.signatory(k) for k in range(S)), np.uint8).reshape(S, 32))
        b = Batch.from_lists(*[[x[k] for x in rows] for k in range(7)])
        ws = work_stream()
        with torch.cuda.stream(ws):
            db = DeviceBatch.from_host(b)
            dg = torch.from_numpy(np.frombuffer(b"".join(digests), np.uint8).reshape(-1, 32).copy()).cuda()
            n = len(rows)
            for rnd in range(3):
                vd = torch.full((n,), 9, dtype=torch.uint8, device="cuda")
                rec = torch.zeros((n, 32), dtype=torch.uint8, device="cuda")
                verify_digest_device(v, db, dg, vd.data_ptr(), rec.data_ptr(), stream=ws)
                ws.synchronize()
                assert vd.cpu().tolist() == want, rnd
                assert rec.cpu().numpy().tobytes() == b"".join(wrec), rnd
                if rnd > 0:
                    assert v.fastpath_stats()[1] == n // 2, rnd   # only the mismatching Froms fall back
    finally:
        v.close()
