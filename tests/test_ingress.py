"""End-to-end batch ingress on the GPU (hyperdrive_amd/ingress.py): wire bytes
-> unmarshal -> verify -> filterHeight -> mq -> consume(current height) ->
vote logs, against the chain of CPU restatements: surge_codec (message.go
Marshal/Unmarshal), the C oracle's verification (libsecp256k1 semantics),
mq_oracle (mq.go) and votes_oracle (process.go logs).

The workload is the seeded adversarial generator (30 % invalid across the C5
classes) over many heights, plus re-sent duplicates and double votes, so
every branch of the chain is exercised: invalid verdicts dropped, heights
below the current one filtered, future heights buffered, per-sender
capacity truncation, first-wins / duplicate / double-vote statuses."""
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
    adm = {sigs[k].tobytes(): k for k in range(S)}
    ing = Ingress(verifier, height=H0, max_capacity=cap)
    try:
        _run(ing, hb, order, sigs, adm, H0, cap, coracle)
    finally:
        ing.close()


def _run(ing, hb, order, sigs, adm, H0, cap, coracle):
    import torch
    mq = MQO.MessageQueue(cap)
    arrival = []
    for t in (2, 3):
        idx = order[hb.type[order] == t]
        buf = SC.marshal_array(t, hb.height[idx], hb.round[idx], None, hb.value[idx], hb.frm[idx], hb.sig[idx])
        d = torch.frombuffer(bytearray(buf), dtype=torch.uint8).cuda()
        vg = ing.push_wire(t, d, len(idx)).cpu().numpy()
        from hyperdrive_amd.verify import Batch
        sub = Batch(hb.type[idx], hb.height[idx], hb.round[idx], None, hb.value[idx], hb.frm[idx], hb.sig[idx])
        vc, _ = coracle.verify(sub, sigs, True, threads=8)
        assert vg.tolist() == vc.tolist()
        for k, i in enumerate(idx):
            if vc[k] == 0 and hb.height[i] >= H0:
                mq.insert(adm[hb.frm[i].tobytes()], _rows(hb, [i])[0])
        arrival += list(idx)
    assert len(ing.mq) == len(mq)
    votes = VO.VoteLogs(H0)
    for step in range(3):
        h = H0 + step
        if step:
            ing.reset_height(h)
            mq.drop_below(h)
            votes.reset(h)
        res = ing.flush()
        n_o, want = mq.consume(h)
        got = [(int(res.senders[k]), r) for k, r in enumerate(_rows(res.consumed, range(len(res.consumed))))]
        assert got == want and len(res.consumed) == n_o
        for k, (s, m) in enumerate(want):
            st, _ = votes.insert(m[2], m[0], m[1], m[4], m[5])
            assert res.vote_status[k] == st
        for t in (2, 3):
            for r in range(4):
                assert ing.votes.len(t, r) == votes.len(t, r)
                for (s, m) in want:
                    assert ing.votes.count(t, r, m[4]) == votes.count(t, r, m[4])
        assert len(want) > 0
