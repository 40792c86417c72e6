"""GPU tally (hd_tally / hd_tally_device_bitmap, through the C ABI) against the
oracle's restatement of process.go's first-wins logs and count loops
(process.go:823-892; 486-494, 534, 574-582, 626-632, 658, 696-702, 751).

Cases: the process_test-style threshold scenarios (tests/tally_cases.py), a
C5-style 64k adversarial batch with duplicates and double votes, the C3
shape (1000 signatories, 64 rounds, proposes interleaved), a heavy-collision
batch (few rounds, many duplicates) and the empty / no-candidate edges."""
import numpy as np
import pytest

from hyperdrive_amd import quorum
from tally_cases import scenarios
from util import from_np, to_np

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def verifier(gpu):
    v = gpu.Verifier(0)
    yield v
    v.close()


def _same(tal, ot):
    assert tal.count == ot.count
    assert tal.distinct == ot.distinct
    assert tal.distinct_any == ot.distinct_any
    assert tal.dup.tolist() == ot.dup


@pytest.mark.parametrize("sc", scenarios(), ids=lambda s: s.name)
def test_scenarios_match_oracle(verifier, oracle, sc):
    b = to_np(sc.b)
    verdicts = np.array(sc.verdicts(), np.uint8)
    tal = verifier.tally(b, verdicts)
    ot = oracle.tally(sc.b, sc.verdicts())
    _same(tal, ot)
    for h, r, pvalue, pvalid, want in sc.expect:
        got = quorum.decide(tal, h, r, sc.f, pvalue, pvalid)
        assert got == oracle.decide_round(ot, h, r, sc.f, pvalue, pvalid)
        for k, v in want.items():
            assert got[k] == v, (sc.name, k)


@pytest.mark.parametrize("kind,n,S,adv", [(0, 65536, 100, 30), (1, 128064, 1000, 10)])
def test_generated_batches_match_oracle(verifier, oracle, coracle, kind, n, S, adv):
    """GPU verify -> GPU tally == oracle tally over the same verdicts; the
    C3 shape (kind 1) is the 1000-signatory, 64-round config.  Every GPU
    verdict and recovered signatory of the batch is the C oracle's too, on the
    full-recovery pass and on the known-key pass (process.go:823-892 consumes
    exactly these verdicts)."""
    from hyperdrive_amd.device import generate
    ks = verifier.gen_keys(S)
    verifier.set_signatories(ks[0])
    db, _, _ = generate(verifier, kind, n, S, adv, keys=ks)
    hb = db.to_host()
    cv, crec = coracle.verify(hb, ks[0], True, threads=16)
    for _ in range(2):      # the first pass learns the keys, the second checks with them
        res, tal = verifier.process_batch(hb)
        assert res.verdict.tolist() == cv.tolist()
        assert res.recovered.tobytes() == crec.tobytes()
    assert (cv == 0).sum() > n // 2
    ot = oracle.tally(from_np(hb), res.verdict.tolist())
    _same(tal, ot)
    f = quorum.thresholds(S)[0]
    for (h, r) in list(ot.distinct_any)[:50]:
        pv = oracle.canonical_value(h, r)
        assert quorum.decide(tal, h, r, f, pv, True) == oracle.decide_round(ot, h, r, f, pv, True)


def test_dense_and_hashed_logs(verifier, oracle):
    """Half the signers admitted: their logs take the dense cells, the others
    the hashed table, inside one tally (a VALID verdict for a From outside
    the context's current set, as after a set change) -- same as the oracle."""
    rng = np.random.default_rng(11)
    n = 8000
    sigs = [oracle.sha256(b"m" + bytes([k])) for k in range(40)]
    vals = [oracle.sha256(b"w" + bytes([k])) for k in range(3)]
    ob = oracle.Batch()
    for i in range(n):
        ob.append(int(rng.integers(2, 4)), int(rng.integers(0, 3)), int(rng.integers(0, 3)), -1,
                  vals[int(rng.integers(0, 3))], sigs[int(rng.integers(0, 40))], bytes(65))
    verdicts = [oracle.VALID if rng.random() < 0.95 else oracle.BAD_RS for _ in range(n)]
    verifier.set_signatories(np.frombuffer(b"".join(sigs[:20]), np.uint8).reshape(20, 32))
    tal = verifier.tally(to_np(ob), np.array(verdicts, np.uint8))
    _same(tal, oracle.tally(ob, verdicts))


def test_heavy_collisions(verifier, oracle):
    """3 rounds, 40 signers, every signer votes ~25 times per (round, type) with
    a few values: long probe chains in every table, most votes duplicates."""
    rng = np.random.default_rng(7)
    n = 6000
    sigs = [oracle.sha256(b"c" + bytes([k])) for k in range(40)]
    vals = [oracle.sha256(b"v" + bytes([k])) for k in range(3)] + [bytes(32)]
    ob = oracle.Batch()
    for i in range(n):
        ob.append(int(rng.integers(2, 4)), int(rng.integers(0, 2)), int(rng.integers(0, 2)), -1,
                  vals[int(rng.integers(0, 4))], sigs[int(rng.integers(0, 40))], bytes(65))
    verdicts = [oracle.VALID if rng.random() < 0.9 else oracle.BAD_RS for _ in range(n)]
    tal = verifier.tally(to_np(ob), np.array(verdicts, np.uint8))
    _same(tal, oracle.tally(ob, verdicts))


def test_no_candidates_and_single(verifier, oracle):
    ob = oracle.Batch()
    for t in (1, 2, 3):
        ob.append(t, 1, 0, -1, bytes(32), oracle.sha256(b"x"), bytes(65))
    verdicts = [oracle.VALID, oracle.BAD_RS, oracle.NOT_ADMITTED]     # a propose is never a candidate
    tal = verifier.tally(to_np(ob), np.array(verdicts, np.uint8))
    _same(tal, oracle.tally(ob, verdicts))
    assert tal.count == {} and tal.distinct_any == {}
    verdicts = [oracle.VALID] * 3
    tal = verifier.tally(to_np(ob), np.array(verdicts, np.uint8))
    _same(tal, oracle.tally(ob, verdicts))


def test_bitmap_entry_equals_verdict_entry(verifier, oracle):
    """hd_tally_device_bitmap (the multi-GPU path after the all-gather) gives
    the same tally as hd_tally on the verdicts."""
    import ctypes
    import torch
    from hyperdrive_amd import _lib
    from hyperdrive_amd.device import generate, work_stream
    n, S = 8192, 50
    ks = verifier.gen_keys(S)
    verifier.set_signatories(ks[0])
    db, _, _ = generate(verifier, 0, n, S, 40, keys=ks)
    hb = db.to_host()
    res = verifier.verify_batch(hb)
    ref = verifier.tally(hb, res.verdict)
    bm = torch.from_numpy(res.valid_bitmap.view(np.int32)).cuda()
    t, a = verifier._tally_struct(n)
    lib = _lib.load()
    cs = db.c_struct()
    torch.cuda.synchronize()
    rc = lib.hd_tally_device_bitmap(verifier.handle, ctypes.byref(cs), bm.data_ptr(), ctypes.byref(t),
                                    work_stream().cuda_stream)
    assert rc == 0
    got = verifier._tally_result(hb, t, a)
    assert got.count == ref.count and got.distinct == ref.distinct and got.distinct_any == ref.distinct_any
    assert got.dup.tolist() == ref.dup.tolist()


@pytest.mark.parametrize("kind,n,S,adv", [(0, 65536, 100, 30), (1, 128064, 1000, 10)])
def test_partitioned_tally_merges_to_the_whole(verifier, kind, n, S, adv):
    """hd_tally_device_bitmap_part over nparts = 2, 3 and 8 partitions of the
    rounds (what each of G ranks runs after the bitmap all-gather): the
    partitions' rows are disjoint, their merge in first-batch-index order is
    exactly the unpartitioned tally (count and round tables, hr_rep
    included), the min-merged dup flags equal its dup, and every row sits in
    the partition hd_tally_partition_of names."""
    import ctypes
    import torch
    from hyperdrive_amd import _lib
    from hyperdrive_amd.device import generate, work_stream
    from hyperdrive_amd.shard import merge_tally_parts, pack_tally, partition_of
    ks = verifier.gen_keys(S)
    verifier.set_signatories(ks[0])
    db, _, _ = generate(verifier, kind, n, S, adv, keys=ks)
    hb = db.to_host()
    res = verifier.verify_batch(hb)
    bm = torch.from_numpy(res.valid_bitmap.view(np.int32)).cuda()
    lib = _lib.load()
    cs = db.c_struct()
    ws = work_stream().cuda_stream
    torch.cuda.synchronize()
    t, a = verifier._tally_struct(n)
    assert lib.hd_tally_device_bitmap(verifier.handle, ctypes.byref(cs), bm.data_ptr(), ctypes.byref(t), ws) == 0
    whole = pack_tally(a, t.n_counts, t.n_hr)
    whole_dup = a["dup"][:n].copy()
    for nparts in (2, 3, 8):
        parts, dup = [], np.full(n, 3, np.uint8)
        for p in range(nparts):
            t, a = verifier._tally_struct(n)
            assert lib.hd_tally_device_bitmap_part(verifier.handle, ctypes.byref(cs), bm.data_ptr(), p, nparts,
                                                   ctypes.byref(t), ws) == 0
            part = pack_tally(a, t.n_counts, t.n_hr)
            for row in part["hr"][:20]:
                assert partition_of(row[0], row[1], nparts) == p
            parts.append(part)
            dup = np.minimum(dup, a["dup"][:n])
        merged = merge_tally_parts(parts)
        assert np.array_equal(merged["counts"], whole["counts"]), nparts
        assert np.array_equal(merged["hr"], whole["hr"]), nparts
        assert np.array_equal(dup, whole_dup), nparts
        assert sum(len(p["hr"]) for p in parts) == len(whole["hr"])


@pytest.mark.parametrize("kind,n,S,adv", [(0, 65536, 100, 30), (1, 128064, 1000, 10)])
def test_async_tally_equals_sync(gpu, kind, n, S, adv):
    """hd_tally_device_bitmap_async + hd_tally_collect give exactly what
    hd_tally_device_bitmap gives (rows, counts, classification), including the
    first submit on a fresh context, whose staged capacity is too small for
    these batches: collect returns HD_EAGAIN and raises the guess, and the
    next submit fits.  A stage smaller than hd_tally_stage_bytes is refused
    with HD_ECAP before anything is queued."""
    import ctypes

    import torch
    from hyperdrive_amd import _lib
    from hyperdrive_amd.device import generate, work_stream
    lib = _lib.load()
    v = gpu.Verifier(0)
    stage = ctypes.c_void_p()
    try:
        ks = v.gen_keys(S)
        v.set_signatories(ks[0])
        db, _, _ = generate(v, kind, n, S, adv, keys=ks)
        nn = db.n
        shard = db.c_struct()
        ws = work_stream()
        with torch.cuda.stream(ws):    # the bitmap's fill ordered before the library's kernels
            verdict = torch.empty(nn, dtype=torch.uint8, device="cuda")
            bitmap = torch.zeros((nn + 31) // 32, dtype=torch.int32, device="cuda")
        s = ws.cuda_stream
        for _ in range(2):
            v.verify_batch_device(shard, verdict.data_ptr(), None, None, bitmap.data_ptr(), s)
        torch.cuda.synchronize()
        ref, ra = v._tally_struct(nn, pinned=False)
        assert lib.hd_tally_device_bitmap(v.handle, ctypes.byref(shard), bitmap.data_ptr(), ctypes.byref(ref), s) == 0
        # a fresh context's guesses (1024 groups) are below these batches' counts
        v2 = gpu.Verifier(0)
        try:
            v2.set_signatories(ks[0])
            cap = 64 << 20
            assert lib.hd_host_alloc(cap, ctypes.byref(stage)) == 0
            t = _lib.HdTallyTicket()
            t.stage, t.stage_cap, t.dup = stage.value, 16, 1
            assert lib.hd_tally_device_bitmap_async(v2.handle, ctypes.byref(shard), bitmap.data_ptr(),
                                                    ctypes.byref(t), s) == _lib.HD_ECAP
            assert t.need == lib.hd_tally_stage_bytes(v2.handle, nn, 1) > 16
            rcs = []
            for _ in range(2):
                t.stage_cap = cap
                assert lib.hd_tally_device_bitmap_async(v2.handle, ctypes.byref(shard), bitmap.data_ptr(),
                                                        ctypes.byref(t), s) == 0
                torch.cuda.synchronize()
                got, ga = v2._tally_struct(nn, pinned=False)
                rcs.append(lib.hd_tally_collect(v2.handle, ctypes.byref(t), ctypes.byref(got)))
            assert rcs[0] in (0, _lib.HD_EAGAIN) and rcs[1] == 0, rcs
            if ref.n_counts > 1024:
                assert rcs[0] == _lib.HD_EAGAIN
            assert (got.n_hr, got.n_counts) == (ref.n_hr, ref.n_counts)
            for k in ("count_height", "count_round", "count_type", "count_rep", "count_n"):
                assert ga[k][:ref.n_counts].tolist() == ra[k][:ref.n_counts].tolist(), k
            for k in ("hr_height", "hr_round", "hr_prevotes", "hr_precommits", "hr_any", "hr_rep"):
                assert ga[k][:ref.n_hr].tolist() == ra[k][:ref.n_hr].tolist(), k
            assert ga["dup"][:nn].tolist() == ra["dup"][:nn].tolist()
            assert lib.hd_tally_ticket_release(ctypes.byref(t)) == 0 and not t.done
        finally:
            v2.close()
    finally:
        if stage.value:
            lib.hd_host_free(stage)
        v.close()
