"""The C-ABI multi-GPU path (include/hd_verify.h hd_multi_*,
hyperdrive_amd/multi.py) against the single-context path on the same batches:
verdicts, recovered signatories, the valid bitmap and the merged partitioned
tally are identical.  On a one-GPU box the device list [0] runs the RCCL
exchange (one rank) and [0, 0] / [0, 0, 0] run the copy exchange between
contexts sharing the GPU; an 8-GPU node runs the same code with one rank per
device."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _same(a, b):
    ra, ta = a
    rb, tb = b
    assert ra.verdict.tolist() == rb.verdict.tolist()
    assert ra.recovered.tobytes() == rb.recovered.tobytes()
    assert ra.valid_bitmap.tolist() == rb.valid_bitmap.tolist()
    assert ta.count == tb.count and ta.distinct == tb.distinct and ta.distinct_any == tb.distinct_any
    assert ta.dup.tolist() == tb.dup.tolist()


@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0]])
@pytest.mark.parametrize("kind,n,S,adv", [(0, 65536 + 17, 100, 30), (1, 128064, 1000, 10), (0, 37, 7, 50)])
def test_multi_equals_single(gpu, devices, kind, n, S, adv):
    from hyperdrive_amd.device import generate
    from hyperdrive_amd.multi import MultiVerifier
    v = gpu.Verifier(0)
    ks = v.gen_keys(S)
    v.set_signatories(ks[0])
    db, _, _ = generate(v, kind, n, S, adv, keys=ks)
    hb = db.to_host()
    single = v.process_batch(hb)
    m = MultiVerifier(devices)
    try:
        assert m.uses_rccl == (len(set(devices)) == len(devices))
        m.set_signatories(ks[0])
        for rnd in range(2):                   # pass 2: the per-device known-key tables
            _same(m.process_batch(hb), single)
        assert m.fastpath_stats(0)[0] > 0
    finally:
        m.close()
        v.close()


def test_multi_empty_and_errors(gpu):
    from hyperdrive_amd import _lib
    from hyperdrive_amd.multi import MultiVerifier
    from hyperdrive_amd.verify import Batch
    with pytest.raises(_lib.HDError):
        MultiVerifier([99])
    m = MultiVerifier([0, 0])
    e = Batch(np.zeros(0, np.uint8), np.zeros(0, np.int64), np.zeros(0, np.int64), None,
              np.zeros((0, 32), np.uint8), np.zeros((0, 32), np.uint8), np.zeros((0, 65), np.uint8))
    res, tal = m.process_batch(e)
    assert len(res.verdict) == 0 and tal.count == {}
    m.close()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_routed_kernels_match_restatement(gpu, world, monkeypatch):
    """hd_route_candidates_device / hd_unroute_device / hd_tally_routed_device
    (the C4 data path) on one GPU, every rank's shard in turn: the route rows
    are byte-identical to the restatement (tests/test_multi_rank.py
    route_rows_np), the rebuilt batches and global indices to unroute_np, each
    owner's tally to its restated rows, and the owners' merged tables to the
    single-context tally of the whole batch.  The tally's consistency check
    (HD_TALLY_CHECK) runs inside every tally."""
    import torch
    from test_multi_rank import route_rows_np, routed_tally_rows, tally_rows, unroute_np
    from util import from_np
    from hyperdrive_amd.device import DeviceBatch, generate, work_stream
    from hyperdrive_amd.shard import (merge_tally_parts, route_candidates, shard_range, tally_out,
                                      tally_routed_device, unroute)
    monkeypatch.setenv("HD_TALLY_CHECK", "1")
    v = gpu.Verifier(0)
    # The library's kernels and torch's copies on ONE explicit stream: the
    # rows the library writes are read by torch copies, and the received rows
    # torch.cat builds are read by the library.  (Round 4 passed torch's
    # current stream, whose handle is 0 -- which the ABI reads as the
    # context's own non-blocking stream, unordered with torch's work: the
    # cause of the intermittent owner mismatch)
    ws = work_stream()
    cs = ws.cuda_stream
    try:
        with torch.cuda.stream(ws):
            S, n = 50, 20_000 + 13
            ks = v.gen_keys(S)
            v.set_signatories(ks[0])
            db, _, _ = generate(v, 0, n, S, 30, keys=ks, start=99)
            hb = db.to_host()
            res, whole = v.process_batch(hb)
            ob = from_np(hb)
            verdicts = res.verdict.tolist()
            adm = sorted(bytes(x) for x in ks[0])
            bits = torch.from_numpy(res.valid_bitmap.view(np.int32).copy()).cuda()
            sent = {}
            for k in range(world):
                lo, hi = shard_range(n, k, world)
                sub = DeviceBatch(hi - lo, db.type[lo:hi], db.height[lo:hi], db.round[lo:hi], db.valid_round[lo:hi],
                                  db.value[lo:hi], db.frm[lo:hi], db.sig[lo:hi])
                rows, counts = route_candidates(v, sub.c_struct(), bits.data_ptr() + 4 * (lo // 32), lo, world, cs)
                want, want_counts = route_rows_np(ob, verdicts, lo, hi, world, adm)
                assert counts == want_counts
                got = rows[: sum(counts)].cpu().numpy()
                assert got.tobytes() == want.tobytes()
                off = np.concatenate([[0], np.cumsum(counts)])
                for o in range(world):
                    sent[(k, o)] = rows[off[o]: off[o + 1]]
            parts = []
            for o in range(world):
                # a ~10 ms kernel ahead of the concatenation on the same
                # stream: the library's unroute must still see its rows
                torch.cuda._sleep(20_000_000)
                recv = torch.cat([sent[(k, o)] for k in range(world)]).contiguous()
                rb, gidx = unroute(v, recv, cs)
                rnp = recv.cpu().numpy()
                u = unroute_np(rnp, adm)
                assert rb.type.cpu().tolist() == [x[0] for x in u]
                assert rb.height.cpu().tolist() == [x[1] for x in u]
                assert gidx.cpu().tolist() == [x[5] for x in u]
                local = tally_routed_device(v, rb, gidx, cs, tally_out(v, n, pinned=True), "cpu")
                want = routed_tally_rows(rnp, adm)
                assert local["counts"].tolist() == want["counts"].tolist()
                assert local["hr"].tolist() == want["hr"].tolist()
                parts.append({k: t.numpy() for k, t in local.items()})
            merged = merge_tally_parts(parts)
            single = tally_rows(ob, verdicts)
            assert merged["counts"].tolist() == single["counts"].tolist()
            assert merged["hr"].tolist() == single["hr"].tolist()
            assert sum(merged["counts"][:, 4].tolist()) == sum(whole.count.values())
    finally:
        v.close()


def test_route_refuses_candidates_outside_the_set(gpu):
    """A VALID candidate whose From left the admitted set after verification
    cannot be named by a route row (rows carry the admitted index), so
    hd_route_candidates_device refuses the batch (HD_EINVAL, with the count in
    the context's last error) instead of tallying it under a synthetic From;
    with the set restored the same call routes every candidate."""
    import torch
    from hyperdrive_amd import _lib
    from hyperdrive_amd.device import generate
    from hyperdrive_amd.shard import route_candidates
    from hyperdrive_amd.device import work_stream
    v = gpu.Verifier(0)
    try:
        S, n = 20, 4096
        ks = v.gen_keys(S)
        v.set_signatories(ks[0])
        db, _, _ = generate(v, 0, n, S, 0, keys=ks)
        res = v.verify_batch(db.to_host())
        ws = work_stream()
        with torch.cuda.stream(ws):                 # the library's kernels ordered after the bitmap's upload
            bits = torch.from_numpy(res.valid_bitmap.view(np.int32).copy()).cuda()
        cs = ws.cuda_stream
        v.set_signatories(ks[0][: S // 2])          # half the signers leave
        with pytest.raises(_lib.HDError) as e:
            route_candidates(v, db.c_struct(), bits.data_ptr(), 0, 3, cs)
        assert e.value.code == _lib.HD_EINVAL and "not in the current admitted set" in str(e.value)
        v.set_signatories(ks[0])
        _, counts = route_candidates(v, db.c_struct(), bits.data_ptr(), 0, 3, cs)
        assert sum(counts) == int((res.verdict == 0).sum())
    finally:
        v.close()


def test_multi_error_return_then_routed_tally(gpu, monkeypatch):
    """Teardown order: an hd_multi [0, 0, 0] call that fails late (HD_ECAP
    from the merge, after every device queued its output downloads and ran
    its routed tally) must hand the caller's arrays back drained; destroying
    the hd_multi at once must not leave work that writes into memory a fresh
    context then allocates.  The routed tally on that fresh context equals
    the restatement, with the tally's consistency check on."""
    import ctypes
    import torch
    from test_multi_rank import route_rows_np, routed_tally_rows
    from util import from_np
    from hyperdrive_amd import _lib
    from hyperdrive_amd.device import generate, work_stream
    from hyperdrive_amd.multi import MultiVerifier
    from hyperdrive_amd.shard import route_candidates, tally_out, tally_routed_device, unroute
    from hyperdrive_amd.verify import Verifier, _ptr
    monkeypatch.setenv("HD_TALLY_CHECK", "1")
    v = gpu.Verifier(0)
    try:
        S, n = 50, 30_000 + 7
        ks = v.gen_keys(S)
        v.set_signatories(ks[0])
        db, _, _ = generate(v, 0, n, S, 30, keys=ks, start=7)
        hb = db.to_host()
        res, _ = v.process_batch(hb)
        m = MultiVerifier([0, 0, 0])
        m.set_signatories(ks[0])
        verdict = np.zeros(n, np.uint8)
        rec = np.zeros((n, 32), np.uint8)
        bitmap = np.zeros((n + 31) // 32, np.uint32)
        t, a = Verifier._tally_struct(n)
        t.cap_counts = 1                           # too small: HD_ECAP after the routed tallies
        cb = hb.c_struct()
        rc = m._lib.hd_multi_verify_batch(m._m, ctypes.byref(cb), _ptr(verdict), _ptr(rec), _ptr(bitmap),
                                          ctypes.byref(t))
        assert rc == _lib.HD_ECAP and t.n_counts > 1
        # the downloads queued before the failure have landed
        assert verdict.tolist() == res.verdict.tolist() and rec.tobytes() == res.recovered.tobytes()
        m.close()
        del verdict, rec, bitmap
        # a fresh context routes the whole batch to one owner and tallies it
        v2 = gpu.Verifier(0)
        try:
            v2.set_signatories(ks[0])
            ws = work_stream()
            with torch.cuda.stream(ws):
                bits = torch.from_numpy(res.valid_bitmap.view(np.int32).copy()).cuda()
                rows, counts = route_candidates(v2, db.c_struct(), bits.data_ptr(), 0, 1, ws.cuda_stream)
                adm = sorted(bytes(x) for x in ks[0])
                want_rows, _ = route_rows_np(from_np(hb), res.verdict.tolist(), 0, n, 1, adm)
                recv = rows[: counts[0]]
                assert recv.cpu().numpy().tobytes() == want_rows.tobytes()
                rb, gidx = unroute(v2, recv, ws.cuda_stream)
                local = tally_routed_device(v2, rb, gidx, ws.cuda_stream, tally_out(v2, n, pinned=True), "cpu")
            want = routed_tally_rows(want_rows, adm)
            assert local["counts"].tolist() == want["counts"].tolist()
            assert local["hr"].tolist() == want["hr"].tolist()
        finally:
            v2.close()
    finally:
        v.close()


def test_tally_check_runs_clean(gpu, monkeypatch):
    """HD_TALLY_CHECK=1 runs the tally's consistency kernels (one winner per
    log cell, unique C / D keys, sum of counts == winners) inside
    hd_tally_device_bitmap on the 30 % adversarial mix, including Froms
    outside the admitted set (the hashed log table D), and leaves the results
    unchanged."""
    from hyperdrive_amd.device import generate
    v = gpu.Verifier(0)
    try:
        S, n = 100, 65536 + 5
        ks = v.gen_keys(S)
        v.set_signatories(ks[0])
        db, _, _ = generate(v, 0, n, S, 30, keys=ks)
        hb = db.to_host()
        res, plain = v.process_batch(hb)
        monkeypatch.setenv("HD_TALLY_CHECK", "1")
        _, checked = v.process_batch(hb)
        assert checked.count == plain.count and checked.dup.tolist() == plain.dup.tolist()
        # verdicts from before a set change: VALID Froms now outside the set take D
        v.set_signatories(ks[0][: S // 2])
        t2 = v.tally(hb, res.verdict)
        monkeypatch.delenv("HD_TALLY_CHECK")
        t3 = v.tally(hb, res.verdict)
        assert t2.count == t3.count and t2.dup.tolist() == t3.dup.tolist()
    finally:
        v.close()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_local_tally_plus_shared_rounds_match_restatement(gpu, world, monkeypatch):
    """The default N > 1 tally (bench.Pipeline.tally, shard.py) on one GPU,
    every rank's shard in turn: each shard's own tally equals its restatement
    (reps + lo), the listed route (hd_route_candidates_listed_device: only the
    rounds present in more than one shard) is byte-identical to
    route_rows_np(rounds=...), the owners' tallies of what they received equal
    theirs, and local rows without the shared rounds plus the owners' rows
    merge to the single-context tally.  Heights run in index order (C2/C4),
    so only the rounds a shard boundary cuts are routed."""
    import torch
    from test_multi_rank import local_tally_rows, route_rows_np, routed_tally_rows, tally_rows
    from util import from_np
    from hyperdrive_amd.device import DeviceBatch, generate, work_stream
    from hyperdrive_amd.shard import (drop_rounds, merge_tally_parts, route_candidates, shard_range,
                                      tally_out, tally_part_device, tally_routed_device, unroute)
    monkeypatch.setenv("HD_TALLY_CHECK", "1")
    v = gpu.Verifier(0)
    ws = work_stream()
    cs = ws.cuda_stream
    try:
        with torch.cuda.stream(ws):
            S, n = 50, 20_000 + 13
            ks = v.gen_keys(S)
            v.set_signatories(ks[0])
            db, _, _ = generate(v, 0, n, S, 30, keys=ks, start=99)
            hb = db.to_host()
            res, whole = v.process_batch(hb)
            ob = from_np(hb)
            verdicts = res.verdict.tolist()
            adm = sorted(bytes(x) for x in ks[0])
            bits = torch.from_numpy(res.valid_bitmap.view(np.int32).copy()).cuda()
            subs, locals_ = [], []
            for k in range(world):
                lo, hi = shard_range(n, k, world)
                sub = DeviceBatch(hi - lo, db.type[lo:hi], db.height[lo:hi], db.round[lo:hi], db.valid_round[lo:hi],
                                  db.value[lo:hi], db.frm[lo:hi], db.sig[lo:hi])
                local = tally_part_device(v, sub.c_struct(), bits.data_ptr() + 4 * (lo // 32), 0, 1, cs,
                                          tally_out(v, hi - lo, pinned=True), "cpu")
                local = {key: t.clone() for key, t in local.items()}
                local["counts"][:, 3] += lo
                local["hr"][:, 5] += lo
                want = local_tally_rows(ob, verdicts, lo, hi)
                assert local["counts"].tolist() == want["counts"].tolist()
                assert local["hr"].tolist() == want["hr"].tolist()
                subs.append((lo, hi, sub))
                locals_.append(local)
            seen = {}
            for local in locals_:
                for h, r in {(int(a), int(b)) for a, b in local["hr"][:, :2].tolist()}:
                    seen[(h, r)] = seen.get((h, r), 0) + 1
            shared_set = {key for key, c in seen.items() if c > 1}
            assert 1 <= len(shared_set) <= 2 * (world - 1)
            shared = torch.tensor(sorted(shared_set), dtype=torch.int64).reshape(-1, 2).cuda()
            sent = {}
            for k, (lo, hi, sub) in enumerate(subs):
                rows, counts = route_candidates(v, sub.c_struct(), bits.data_ptr() + 4 * (lo // 32), lo, world, cs,
                                                rounds=shared)
                want_rows, want_counts = route_rows_np(ob, verdicts, lo, hi, world, adm, rounds=shared_set)
                assert counts == want_counts
                assert rows[: sum(counts)].cpu().numpy().tobytes() == want_rows.tobytes()
                off = np.concatenate([[0], np.cumsum(counts)])
                for o in range(world):
                    sent[(k, o)] = rows[off[o]: off[o + 1]]
            parts = []
            for o in range(world):
                recv = torch.cat([sent[(k, o)] for k in range(world)]).contiguous()
                mine = {key: drop_rounds(t, shared.cpu()) for key, t in locals_[o].items()}
                if recv.shape[0]:
                    rb, gidx = unroute(v, recv, cs)
                    own = tally_routed_device(v, rb, gidx, cs, tally_out(v, n, pinned=True), "cpu")
                    want = routed_tally_rows(recv.cpu().numpy(), adm)
                    assert own["counts"].tolist() == want["counts"].tolist()
                    mine = {key: torch.cat([mine[key], own[key]]) for key in mine}
                parts.append({key: t.numpy() for key, t in mine.items()})
            merged = merge_tally_parts(parts)
            single = tally_rows(ob, verdicts)
            assert merged["counts"].tolist() == single["counts"].tolist()
            assert merged["hr"].tolist() == single["hr"].tolist()
    finally:
        v.close()
