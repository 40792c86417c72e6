"""End-to-end batch ingress on the GPU (hyperdrive_amd/ingress.py): wire bytes
-> unmarshal -> verify -> filterHeight -> mq -> consume(current height) ->
vote logs, against the chain of CPU restatements: surge_codec (message.go
Marshal/Unmarshal), the C oracle's verification (libsecp256k1 semantics),
mq_oracle (mq.go) and votes_oracle (process.go logs).

The workload is the seeded adversarial generator (30 % invalid across the C5
classes) over many heights, plus re-sent duplicates and double votes, so
every branch of the chain is exercised: invalid verdicts dropped, heights
below the current one filtered, future heights buffered, per-sender
capacity truncation, first-wins / duplicate / double-vote statuses.

Membership is the reference's: the restatement chain inserts
every AUTHENTICATED message (the C oracle's verdict VALID or NOT_ADMITTED:
recovered signatory == From) into mq_oracle keyed by From, and applies
procsAllowed only in mq_oracle.consume(allowed=...) (mq.go:49-51).  The
admitted set starts at five of the seven signers and is replaced mid-stream
by a ResetHeight with a new signatory set (replica.go:132-145): messages
buffered from the two signers admitted only then are delivered after it,
those of the signers it removes are dropped at consume."""
import numpy as np
import pytest

import mq_oracle as MQO
import surge_codec as SC
import votes_oracle as VO

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def verifier(gpu):
    v = gpu.Verifier(0)
    yield v
    v.close()


def _rows(b, idx):
    return [(int(b.height[i]), int(b.round[i]), int(b.type[i]), int(b.valid_round[i]) if b.type[i] == 1 else -1,
             b.value[i].tobytes(),
             b.frm[i].tobytes(), b.sig[i].tobytes()) for i in idx]


@pytest.mark.parametrize("cap", [1000, 4])
def test_wire_to_vote_logs_matches_restatements(verifier, coracle, cap):
    import torch
    from hyperdrive_amd.device import generate
    from hyperdrive_amd.ingress import Ingress
    S, n = 7, 1500
    db, sigs, _ = generate(verifier, 0, n, S, adv_pct=30, start=777)
    verifier.set_signatories(sigs)
    hb = db.to_host()
    H0 = int(np.median(hb.height))          # heights below are filtered, above buffered
    # 200 messages are re-sent later in the stream: VALID again, buffered
    # again by mq, then logged as identical duplicates
    rng = np.random.default_rng(cap)
    extra = rng.choice(n, 200, replace=False)
    # arrival with heights shuffled by up to +-50: out-of-order
    # heights reach mq, which must restore (height, round, arrival) order
    jitter = np.arange(n) + rng.integers(-50, 51, n) * 2 * S
    order = np.concatenate([np.argsort(jitter, kind="stable"), extra])
    # arrival = per-type wire buffers pushed in this order: prevotes, precommits
    first, later = sigs[:5], sigs[2:]        # admitted sets before / after the ResetHeight
    verifier.set_signatories(first)
    ing = Ingress(verifier, height=H0, max_capacity=cap)
    try:
        _run(ing, hb, order, first, later, H0, cap, coracle)
    finally:
        ing.close()


def _run(ing, hb, order, first, later, H0, cap, coracle):
    import torch
    from hyperdrive_amd.verify import Batch
    mq = MQO.MessageQueue(cap)
    for t in (2, 3):
        idx = order[hb.type[order] == t]
        buf = SC.marshal_array(t, hb.height[idx], hb.round[idx], None, hb.value[idx], hb.frm[idx], hb.sig[idx])
        d = torch.frombuffer(bytearray(buf), dtype=torch.uint8).cuda()
        vg = ing.push_wire(t, d, len(idx)).cpu().numpy()
        sub = Batch(hb.type[idx], hb.height[idx], hb.round[idx], None, hb.value[idx], hb.frm[idx], hb.sig[idx])
        vc, _ = coracle.verify(sub, first, True, threads=8)
        # authenticate_batch_device: VALID / NOT_ADMITTED exactly the oracle's,
        # every other message the oracle's verdict or NOT_AUTHENTIC (8)
        auth_c = np.isin(vc, (0, 6))
        assert (vg[auth_c] == vc[auth_c]).all() and not np.isin(vg[~auth_c], (0, 6)).any()
        assert ((vg[~auth_c] == vc[~auth_c]) | (vg[~auth_c] == 8)).all()
        assert (vc == 6).sum() > 0              # authenticated senders outside the admitted set
        for k, i in enumerate(idx):
            # authenticated (VALID or NOT_ADMITTED) and filterHeight: mq.Insert*
            if vc[k] in (0, 6) and hb.height[i] >= H0:
                mq.insert(hb.frm[i].tobytes(), _rows(hb, [i])[0])
    assert len(ing.mq) == len(mq)
    votes = VO.VoteLogs(H0)
    allowed = {x.tobytes() for x in first}
    ids = {}
    late = {x.tobytes() for x in later} - allowed
    delivered_late = 0
    for step in range(3):
        h = H0 + step
        if step:
            # step 1: ResetHeight with a new signatory set; step 2: without
            sigset = later if step == 1 else None
            ing.reset_height(h, sigset)
            mq.drop_below(h)
            votes.reset(h)
            if sigset is not None:
                allowed = {x.tobytes() for x in sigset}
                assert ing.f == len(sigset) // 3
        res = ing.flush()
        n_o, want = mq.consume(h, allowed=allowed)
        rows = _rows(res.consumed, range(len(res.consumed)))
        assert [(m[5], m) for m in rows] == want and len(res.consumed) == len(want)
        assert res.removed == n_o
        for m, sid in zip(rows, res.senders.tolist()):
            assert ids.setdefault(m[5], sid) == sid
        if step:
            delivered_late += sum(1 for m in rows if m[5] in late)
        for k, (s, m) in enumerate(want):
            st, _ = votes.insert(m[2], m[0], m[1], m[4], m[5])
            assert res.vote_status[k] == st
        for t in (2, 3):
            for r in range(4):
                assert ing.votes.len(t, r) == votes.len(t, r)
                for (s, m) in want:
                    assert ing.votes.count(t, r, m[4]) == votes.count(t, r, m[4])
        assert len(want) > 0
    # messages buffered while their sender was not admitted were delivered
    # after the ResetHeight that admitted it
    assert delivered_late > 0


def test_overlapped_push_equals_serial(verifier):
    """push_wires_begin queues a batch's unmarshal + authentication and
    returns; flushes served meanwhile, then push_finish (filterHeight + mq
    insert at the height reached), deliver exactly what the serial order
    (flushes, then push_wires) delivers: every flush's messages, sender ids,
    vote statuses and removed counts, and the queue afterwards."""
    from hyperdrive_amd.codec import marshal_device
    from hyperdrive_amd.device import DeviceBatch, generate
    from hyperdrive_amd.ingress import Ingress
    S, n = 7, 4000
    db, sigs, _ = generate(verifier, 0, n, S, adv_pct=30, start=4242)
    verifier.set_signatories(sigs)
    H0 = int(db.height.min().item())

    def wires(lo, hi):
        out = []
        for t in (2, 3):
            idx = (db.type[lo:hi] == t).nonzero().flatten() + lo
            sub = DeviceBatch(int(idx.numel()), *(getattr(db, f)[idx].contiguous()
                                                   for f in ("type", "height", "round", "valid_round", "value",
                                                             "frm", "sig")))
            out.append((t, marshal_device(verifier, t, sub, with_sig=True), sub.n))
        return out

    w1, w2 = wires(0, n // 2), wires(n // 2, n)

    def flushes(ing, h0, k):
        res = []
        for h in range(h0, h0 + k):
            if h > ing.height:
                ing.reset_height(h)
            f = ing.flush()
            res.append((f.consumed.height.tolist(), f.consumed.frm.tobytes(), f.consumed.sig.tobytes(),
                        f.senders.tolist(), f.vote_status.tolist(), f.removed))
        return res

    serial, overlapped = Ingress(verifier, height=H0), Ingress(verifier, height=H0)
    try:
        serial.push_wires(w1)
        a = flushes(serial, H0, 6)
        serial.push_wires(w2)
        a += flushes(serial, H0 + 6, 6)
        overlapped.push_wires(w1)
        pend = overlapped.push_wires_begin(w2)
        b = flushes(overlapped, H0, 6)
        overlapped.push_finish(pend)
        b += flushes(overlapped, H0 + 6, 6)
        assert a == b
        assert sum(len(x[0]) for x in a) > 0
        assert len(serial.mq) == len(overlapped.mq)
    finally:
        serial.close()
        overlapped.close()
