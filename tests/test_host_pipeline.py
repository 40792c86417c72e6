"""Asynchronous host-buffer verification (include/hd_verify.h hd_verify_submit /
hd_verify_wait; the cgo caller's path, replica/replica.go:156-181) against the
synchronous hd_verify_batch on the same batches: several tickets in flight
over the context's two pipelines, pageable and pinned inputs and outputs,
golden fixtures -- every verdict, signatory and bitmap word identical."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _pinned_like(a):
    import torch
    t = torch.empty(a.shape, dtype={np.uint8: torch.uint8, np.int64: torch.int64, np.uint16: torch.int16,
                                     np.uint32: torch.int32}[a.dtype.type], pin_memory=True)
    out = t.numpy().view(a.dtype)
    out[...] = a
    return out, t


def test_submit_wait_equals_sync_verify(gpu):
    from hyperdrive_amd.device import generate
    from hyperdrive_amd.verify import Batch
    v = gpu.Verifier(0)
    try:
        S, n = 64, 40_000 + 7
        ks = v.gen_keys(S)
        v.set_signatories(ks[0])
        db, _, _ = generate(v, 0, n, S, 30, keys=ks, start=5)
        hb = db.to_host()
        ref = v.verify_batch(hb)                   # also teaches the context the keys
        ref = v.verify_batch(hb)
        keep = []
        pb = Batch(*[(_pinned_like(a)[0] if a is not None else None) for a in
                     (hb.type, hb.height, hb.round, hb.valid_round, hb.value, hb.frm, hb.sig)])
        outs, tickets = [], []
        for k in range(5):
            src = pb if k % 2 else hb                                # pinned / pageable inputs
            verdict = np.zeros(n, np.uint8)
            rec = np.zeros((n, 32), np.uint8)
            bits = np.zeros((n + 31) // 32, np.uint32)
            if k == 3:                                               # pinned outputs
                (verdict, t1), (rec, t2), (bits, t3) = (_pinned_like(verdict), _pinned_like(rec),
                                                        _pinned_like(bits))
                keep += [t1, t2, t3]
            tickets.append(v.submit(src, verdict, rec, bits))
            outs.append((verdict, rec, bits))
        assert tickets == sorted(tickets) and tickets[0] >= 1
        for t in reversed(tickets):                                  # any order; earlier ones completed by reuse
            v.wait(t)
        v.wait(tickets[0])                                           # completed: returns at once
        for verdict, rec, bits in outs:
            assert verdict.tolist() == ref.verdict.tolist()
            assert rec.tobytes() == ref.recovered.tobytes()
            assert bits.tolist() == ref.valid_bitmap.tolist()
        assert (ref.verdict == 0).sum() > 0 and (ref.verdict != 0).sum() > 0
        from hyperdrive_amd import _lib
        with pytest.raises(_lib.HDError):
            v.wait(0)
    finally:
        v.close()


def test_submit_golden_fixtures(gpu):
    from test_golden import CASES, load_case
    for name in CASES:
        b, z, _ = load_case(name)
        v = gpu.Verifier(0, compressed=int(z["compressed"]))
        try:
            v.set_signatories(z["admitted"])
            n = len(b)
            got = []
            for _ in range(2):                                       # full recovery, then the known-key check
                verdict = np.zeros(n, np.uint8)
                rec = np.zeros((n, 32), np.uint8)
                t = v.submit(b, verdict, rec, None)
                v.wait(t)
                got.append((verdict, rec))
            for verdict, rec in got:
                assert verdict.tolist() == z["verdict"].tolist(), name
                assert rec.tobytes() == z["recovered"].tobytes(), name
        finally:
            v.close()


def test_submit_compact_equals_full(gpu):
    """hd_verify_submit_compact (From / value as 16-bit indices, escape rows
    for senders outside the set) gives byte-identical outputs to
    hd_verify_submit on the expanded batch: the 30 % adversarial mix (its
    foreign senders are escape rows), pinned and pageable, two in flight."""
    from hyperdrive_amd.device import generate
    from hyperdrive_amd.verify import Batch, CompactBatch
    from hyperdrive_amd import _lib
    v = gpu.Verifier(0)
    try:
        S, n = 100, 50_000 + 3
        ks = v.gen_keys(S)
        v.set_signatories(ks[0])
        db, _, _ = generate(v, 0, n, S, 30, keys=ks, start=11)
        hb = db.to_host()
        ref = v.verify_batch(hb)
        ref = v.verify_batch(hb)
        cb = CompactBatch.from_batch(hb, ks[0])
        assert len(cb.escape) > 0 and len(cb.values) > 1
        pcb = CompactBatch(*[(_pinned_like(a)[0] if a is not None else None) for a in
                             (cb.type, cb.height, cb.round, cb.valid_round, cb.from_idx, cb.value_idx, cb.sig,
                              cb.escape, cb.values)])
        outs, tickets = [], []
        for k in range(4):
            verdict = np.zeros(n, np.uint8)
            rec = np.zeros((n, 32), np.uint8)
            bits = np.zeros((n + 31) // 32, np.uint32)
            tickets.append(v.submit_compact(pcb if k % 2 else cb, verdict, rec, bits))
            outs.append((verdict, rec, bits))
        for t in tickets:
            v.wait(t)
        for verdict, rec, bits in outs:
            assert verdict.tolist() == ref.verdict.tolist()
            assert rec.tobytes() == ref.recovered.tobytes()
            assert bits.tolist() == ref.valid_bitmap.tolist()
        # an index that names no row is refused, nothing queued
        bad = CompactBatch(cb.type, cb.height, cb.round, cb.valid_round, cb.from_idx.copy(), cb.value_idx, cb.sig,
                           cb.escape, cb.values)
        bad.from_idx[17] = S + len(cb.escape)
        with pytest.raises(_lib.HDError):
            v.submit_compact(bad, np.zeros(n, np.uint8))
        bad = CompactBatch(cb.type, cb.height, cb.round, cb.valid_round, cb.from_idx, cb.value_idx.copy(), cb.sig,
                           cb.escape, cb.values)
        bad.value_idx[0] = len(cb.values)
        with pytest.raises(_lib.HDError):
            v.submit_compact(bad, np.zeros(n, np.uint8))
    finally:
        v.close()


def test_submit_compact_golden_fixtures(gpu):
    """every golden fixture through the compact form (full recovery, then the
    known-key check): the fixture's verdicts and recovered signatories"""
    from test_golden import CASES, load_case
    from hyperdrive_amd.verify import CompactBatch
    for name in CASES:
        b, z, _ = load_case(name)
        if len(b) == 0:
            continue
        v = gpu.Verifier(0, compressed=int(z["compressed"]))
        try:
            v.set_signatories(z["admitted"])
            cb = CompactBatch.from_batch(b, z["admitted"])
            n = len(b)
            for _ in range(2):
                verdict = np.zeros(n, np.uint8)
                rec = np.zeros((n, 32), np.uint8)
                v.wait(v.submit_compact(cb, verdict, rec, None))
                assert verdict.tolist() == z["verdict"].tolist(), name
                assert rec.tobytes() == z["recovered"].tobytes(), name
        finally:
            v.close()
