"""Bulk MessageQueue (include/hd_mq.h) against the one-message-at-a-time
restatement of mq/mq.go (oracle/mq_oracle.py).

CPU: the restatement reproduces the reference's own mq_test.go behaviours --
max capacity 1 (mq_test.go:642-714), excess dropped (716-793), ordering by
height and round (334-608), drop below height (611-639), procsAllowed at
consume (119-331).
GPU: queues are keyed by From (the 32 bytes, mq.go:107-113) and procsAllowed
is applied at consume time (mq.go:49-51).  Random insert / consume (with
random procsAllowed subsets) / drop sequences give exactly the restatement's
delivered messages (all fields, order included) and its Consume count n, for
capacities 1, 3, 25 and 1000; the four whitelist scenarios of
mq_test.go:119-331 (allowed, not allowed, removed later, added later) run
through the GPU queue; a 1M-message batch from 100 senders keeps every
sender's 1000 smallest (height, round, arrival) messages."""
import random

import numpy as np
import pytest

from mq_oracle import MessageQueue as OracleMQ


def _msg(h, r, tag=0):
    return (h, r, tag)


def test_oracle_capacity_one():
    # mq_test.go:642-714
    q = OracleMQ(1)
    q.insert("A", _msg(1, 1, "orig"))
    q.insert("B", _msg(1, 2, "b"))
    n, out = q.consume(1)
    assert n == 2 and [m[2] for _, m in out] == ["orig", "b"]
    q.insert("A", _msg(1, 1, "orig"))
    q.insert("A", _msg(1, 2, "late"))          # dropped: queue full, larger key
    n, out = q.consume(1)
    assert n == 1 and out[0][1][2] == "orig"
    q.insert("A", _msg(1, 1, "orig"))
    q.insert("A", _msg(1, 0, "early"))         # evicts the original
    n, out = q.consume(1)
    assert n == 1 and out[0][1][2] == "early"


def test_oracle_drops_excess():
    # mq_test.go:716-793
    rng = random.Random(3)
    for _ in range(20):
        c = 5 + rng.randrange(20)
        q = OracleMQ(c)
        count = c + 5 + rng.randrange(20)
        rounds = list(range(count))
        rng.shuffle(rounds)
        for r in rounds:
            q.insert("s", _msg(1, r))
        n, out = q.consume(1)
        assert n == c and sorted(m[1] for _, m in out) == list(range(c))


def test_oracle_order_stable_and_drop_below():
    rng = random.Random(4)
    q = OracleMQ(1000)
    msgs = [_msg(rng.randrange(5), rng.randrange(3), i) for i in range(200)]
    for m in msgs:
        q.insert("s", m)
    q.drop_below(2)                                   # mq_test.go:611-639
    n, out = q.consume(3)
    got = [m for _, m in out]
    want = sorted([m for m in msgs if 2 <= m[0] <= 3], key=lambda m: (m[0], m[1], m[2]))
    assert got == want and n == len(want)


def test_oracle_procs_allowed_at_consume():
    q = OracleMQ(10)
    q.insert("in", _msg(1, 0))
    q.insert("out", _msg(1, 0))
    n, out = q.consume(1, allowed={"in"})
    assert n == 2 and [s for s, _ in out] == ["in"]


def test_oracle_whitelist_changes_between_consumes():
    # mq_test.go:207-331: removed from / added to procsAllowed between two consumes
    q = OracleMQ(1000)
    q.insert("s", _msg(5, 0, "low"))
    q.insert("s", _msg(9, 0, "high"))
    n, out = q.consume(5, allowed={"s"})
    assert n == 1 and [m[2] for _, m in out] == ["low"]
    n, out = q.consume(9, allowed=set())
    assert n == 1 and out == []
    q.insert("t", _msg(5, 0, "a"))
    q.insert("t", _msg(9, 0, "b"))
    n, out = q.consume(5, allowed=set())
    assert n == 1 and out == []
    n, out = q.consume(9, allowed={"t"})
    assert n == 1 and [m[2] for _, m in out] == ["b"]


def test_oracle_queue_creation_order():
    q = OracleMQ(10)
    for s in ("c", "a", "b"):
        q.insert(s, _msg(1, 0))
    q.consume(1)
    q.insert("a", _msg(2, 0))
    q.insert("d", _msg(2, 0))
    q.insert("c", _msg(2, 0))
    n, out = q.consume(2)
    assert [s for s, _ in out] == ["c", "a", "d"]


# ---------------------------------------------------------------- GPU
@pytest.fixture(scope="module")
def verifier(gpu):
    v = gpu.Verifier(0)
    yield v
    v.close()


def _senders(rng, S):
    return rng.integers(0, 256, (S, 32), dtype=np.uint8)


def _batch(rng, n, keys, hmax, rmax, skip_pct=10):
    """Random messages from the senders `keys` (S x 32 Froms); ~skip_pct %
    are not inserted (insert flag 0)."""
    import torch
    from hyperdrive_amd.device import DeviceBatch
    typ = rng.integers(1, 4, n).astype(np.uint8)
    h = rng.integers(0, hmax, n).astype(np.int64)
    r = rng.integers(0, rmax, n).astype(np.int64)
    vr = rng.integers(-1, 3, n).astype(np.int64)
    value = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    frm = keys[rng.integers(0, len(keys), n)]
    sig = rng.integers(0, 256, (n, 65), dtype=np.uint8)
    ins = (rng.random(n) >= skip_pct / 100).astype(np.uint8)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    db = DeviceBatch(n, t(typ), t(h), t(r), t(vr), t(value), t(frm), t(sig))
    host = [(int(h[i]), int(r[i]), int(typ[i]), int(vr[i]), value[i].tobytes(), frm[i].tobytes(), sig[i].tobytes())
            for i in range(n)]
    return db, t(ins), host, ins


def _rows(b):
    return [(int(b.height[k]), int(b.round[k]), int(b.type[k]), int(b.valid_round[k]), b.value[k].tobytes(),
             b.frm[k].tobytes(), b.sig[k].tobytes()) for k in range(len(b))]


def _check_consumed(b, snd, want, ids):
    """GPU (rows, sender ids) == oracle [(From, row)]; sender ids name the
    queues in creation order (ids: From -> id seen so far, extended here)."""
    rows = _rows(b)
    assert [(m[5], m) for m in rows] == want
    for m, k in zip(rows, snd.tolist()):
        assert ids.setdefault(m[5], k) == k


@pytest.mark.gpu
@pytest.mark.parametrize("cap", [1, 3, 25, 1000])
def test_random_sequences_match_oracle(verifier, cap):
    from hyperdrive_amd.mq import MessageQueue
    rng = np.random.default_rng(cap)
    keys = _senders(rng, 7)
    q = MessageQueue(verifier, cap)
    o = OracleMQ(cap)
    ids = {}
    for step in range(12):
        db, d_ins, host, ins = _batch(rng, int(rng.integers(1, 3000)), keys, 6, 4)
        q.insert_device(db, d_ins)
        for i, m in enumerate(host):
            if ins[i]:
                o.insert(m[5], m)
        assert len(q) == len(o)
        op = step % 3
        if op == 1:
            hh = int(rng.integers(0, 6))
            allowed = keys[rng.random(len(keys)) < 0.6]
            b, s = q.consume(hh, allowed)
            n, want = o.consume(hh, allowed={k.tobytes() for k in allowed})
            _check_consumed(b, s, want, ids)
            assert q.last_removed == n
        elif op == 2:
            hh = int(rng.integers(0, 6))
            q.drop_below(hh)
            o.drop_below(hh)
    # the creation order of the queues is the order of first insertion
    assert sorted(ids.values()) == list(range(len(ids)))
    b, s = q.consume(10 ** 9, keys)
    n, want = o.consume(10 ** 9)
    _check_consumed(b, s, want, ids)
    assert q.senders == len(o.queues)
    q.close()


def _one(h, r, frm, tag):
    import torch
    from hyperdrive_amd.device import DeviceBatch
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    val = np.zeros((1, 32), np.uint8)
    val[0, 0] = tag
    f = np.frombuffer(frm, np.uint8).reshape(1, 32)
    return DeviceBatch(1, t(np.array([1], np.uint8)), t(np.array([h], np.int64)), t(np.array([r], np.int64)),
                       t(np.array([-1], np.int64)), t(val), t(f), t(np.zeros((1, 65), np.uint8)))


@pytest.mark.gpu
def test_capacity_one_on_gpu(verifier):
    """mq_test.go:642-714 through the GPU queue."""
    from hyperdrive_amd.mq import MessageQueue
    A, B = bytes([1]) * 32, bytes([2]) * 32
    q = MessageQueue(verifier, 1)
    q.insert_device(_one(1, 1, A, 1))
    q.insert_device(_one(1, 2, B, 2))
    b, s = q.consume(1, [A, B])
    assert len(b) == 2
    q.insert_device(_one(1, 1, A, 1))
    q.insert_device(_one(1, 2, A, 3))
    b, s = q.consume(1, [A])
    assert len(b) == 1 and b.value[0, 0] == 1
    q.insert_device(_one(1, 1, A, 1))
    q.insert_device(_one(1, 0, A, 4))
    b, s = q.consume(1, [A])
    assert len(b) == 1 and b.value[0, 0] == 4
    q.close()


@pytest.mark.gpu
def test_whitelist_scenarios_on_gpu(verifier):
    """mq_test.go:119-331: the sender whitelisted, not whitelisted, removed
    from and added to procsAllowed between two consumes.  Consume's n counts
    the message either way; only allowed senders' messages are delivered."""
    from hyperdrive_amd.mq import MessageQueue
    rng = np.random.default_rng(5)
    for case in ("allowed", "denied", "removed", "added"):
        for _ in range(4):
            snd = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
            h = int(rng.integers(0, 1 << 62))
            hi = h + 1 + int(rng.integers(0, 100))
            r = int(rng.integers(0, 1 << 62))
            q = MessageQueue(verifier, 1000)
            q.insert_device(_one(h, r, snd, 1))
            if case in ("removed", "added"):
                q.insert_device(_one(hi, r, snd, 2))
            first = [snd] if case in ("allowed", "removed") else []
            b, _ = q.consume(h, first)
            assert q.last_removed == 1 and len(b) == (1 if first else 0)
            if case in ("removed", "added"):
                second = [] if case == "removed" else [snd]
                b, _ = q.consume(hi, second)
                assert q.last_removed == 1 and len(b) == (1 if second else 0)
                if second:
                    assert b.value[0, 0] == 2
            assert len(q) == 0
            q.close()


@pytest.mark.gpu
def test_consume_uses_admitted_set_at_call(gpu):
    """allowed=None is the verifier's admitted set as it is at the consume
    (replica.go:136-143 rebuilds procsAllowed; mq.go:49 reads it then)."""
    from hyperdrive_amd.mq import MessageQueue
    v = gpu.Verifier(0)
    A, B = bytes([7]) * 32, bytes([9]) * 32
    v.set_signatories([A])
    q = MessageQueue(v, 10)
    q.insert_device(_one(1, 0, A, 1))
    q.insert_device(_one(1, 0, B, 2))
    q.insert_device(_one(2, 0, A, 3))
    q.insert_device(_one(2, 0, B, 4))
    b, s = q.consume(1)
    assert b.value[:, 0].tolist() == [1] and q.last_removed == 2
    v.set_signatories([B])
    b, s = q.consume(2)
    assert b.value[:, 0].tolist() == [4] and q.last_removed == 2 and s.tolist() == [1]
    q.close()
    v.close()


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_prefetched_consumes_match_oracle(gpu, seed):
    """Consumes against the admitted set stage the next heights' window
    (hd_mq.hip k_mq_consume1 prefetch) and serve the following consumes on
    the host: every delivery, removed count and queue size still equals the
    oracle through height-by-height flushes, skipped heights, consumes below
    the last one, drops inside and past the window, inserts and admitted-set
    changes between consumes (each of which ends the window)."""
    from hyperdrive_amd.mq import MessageQueue
    rng = np.random.default_rng(100 + seed)
    keys = _senders(rng, 9)
    v = gpu.Verifier(0)
    adm = keys[:6]
    v.set_signatories(adm)
    q = MessageQueue(v, 40)
    o = OracleMQ(40)
    ids = {}
    cur = 0
    for step in range(60):
        op = rng.random()
        if step % 20 == 0 or op < 0.08:
            db, d_ins, host, ins = _batch(rng, int(rng.integers(200, 2000)), keys, cur + 80, 3)
            q.insert_device(db, d_ins)
            for i, m in enumerate(host):
                if ins[i]:
                    o.insert(m[5], m)
        elif op < 0.12:
            adm = keys[rng.random(len(keys)) < 0.6]
            v.set_signatories(adm)
        elif op < 0.2:
            hh = cur + int(rng.integers(-3, 90))
            q.drop_below(hh)
            o.drop_below(hh)
        else:
            r = rng.random()
            cur = cur + (1 if r < 0.7 else int(rng.integers(-5, 20)))
            b, sn = q.consume(cur)
            n, want = o.consume(cur, allowed={k.tobytes() for k in adm})
            _check_consumed(b, sn, want, ids)
            assert q.last_removed == n, step
        assert len(q) == len(o), step
    b, sn = q.consume(10 ** 9)
    n, want = o.consume(10 ** 9, allowed={k.tobytes() for k in adm})
    _check_consumed(b, sn, want, ids)
    assert len(q) == 0
    # admitted-set consumes within the window width of INT64_MAX: the
    # window's end clamps at INT64_MAX instead of overflowing
    top = (1 << 63) - 1
    db, d_ins, host, ins = _batch(rng, 300, keys, 40, 3)
    db.height += top - 40
    q.insert_device(db, d_ins)
    for i, m in enumerate(host):
        if ins[i]:
            o.insert(m[5], (m[0] + top - 40,) + m[1:])
    for hh in (top - 30, top - 29, top - 5, top):
        b, sn = q.consume(hh)
        n, want = o.consume(hh, allowed={k.tobytes() for k in adm})
        _check_consumed(b, sn, want, ids)
        assert q.last_removed == n, hh
        assert len(q) == len(o), hh
    assert len(q) == 0
    q.close()
    v.close()


@pytest.mark.gpu
def test_million_message_insert(verifier):
    """1M messages from 100 senders, cap 1000: every sender keeps its 1000
    smallest (height, round, arrival) messages, in that order."""
    import torch
    from hyperdrive_amd.device import DeviceBatch
    from hyperdrive_amd.mq import MessageQueue
    rng = np.random.default_rng(11)
    n, S = 1 << 20, 100
    h = rng.integers(1, 5000, n).astype(np.int64)
    r = rng.integers(0, 4, n).astype(np.int64)
    snd = (np.arange(n) % S).astype(np.int32)
    keys = _senders(rng, S)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    tag = np.zeros((n, 32), np.uint8)
    tag[:, :4] = np.arange(n, dtype=np.uint32).view(np.uint8).reshape(n, 4)
    db = DeviceBatch(n, t(np.full(n, 2, np.uint8)), t(h), t(r), t(np.full(n, -1, np.int64)), t(tag),
                     t(keys[snd]), t(np.zeros((n, 65), np.uint8)))
    q = MessageQueue(verifier, 1000)
    q.insert_device(db)
    assert len(q) == S * 1000 and q.senders == S
    b, s = q.consume(10 ** 9, keys)
    idx = b.value[:, :4].copy().view(np.uint32).ravel()
    order = np.lexsort((np.arange(n), r, h, snd))           # sender (= creation order), h, r, arrival
    keep = np.concatenate([order[snd[order] == k][:1000] for k in range(S)])
    assert idx.tolist() == keep.tolist()
    assert s.tolist() == snd[keep].tolist()
    q.close()


@pytest.mark.gpu
@pytest.mark.parametrize("cap,S,span", [(1, 50, 1 << 40), (7, 300, 3), (300, 120, 1 << 62), (5, 5000, 100)])
def test_large_inserts_match_restatement(verifier, cap, S, span):
    """Two 70,000-message inserts into one queue (the second merges with the
    sorted pool), heights over a span of 3 (all ties: arrival order decides),
    100, 2^40 and 2^62 (a packed key wider than 64 bits: the three-pass
    sort), 50 to 5,000 senders.  The queue keeps, per sender, the first `cap`
    messages by (height, round, arrival) over both batches together."""
    import torch
    from hyperdrive_amd.device import DeviceBatch
    from hyperdrive_amd.mq import MessageQueue
    rng = np.random.default_rng(cap * 7919 + S)
    keys = _senders(rng, S)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    q = MessageQueue(verifier, cap)
    n = 70000
    hs, rs, ss = [], [], []
    for step in range(2):
        lo = -(span // 2)
        h = (lo + rng.integers(0, span, n)).astype(np.int64)
        r = rng.integers(-1, 3, n).astype(np.int64)
        snd = (np.arange(n) % S) if step == 0 else rng.integers(0, S, n)
        tag = np.zeros((n, 32), np.uint8)
        tag[:, :4] = (np.arange(n, dtype=np.uint32) + step * n).view(np.uint8).reshape(n, 4)
        db = DeviceBatch(n, t(np.full(n, 2, np.uint8)), t(h), t(r), t(np.full(n, -1, np.int64)), t(tag),
                         t(keys[snd]), t(np.zeros((n, 65), np.uint8)))
        q.insert_device(db)
        hs.append(h)
        rs.append(r)
        ss.append(snd)
    h, r, snd = np.concatenate(hs), np.concatenate(rs), np.concatenate(ss)
    order = np.lexsort((np.arange(2 * n), r, h, snd))
    keep = np.concatenate([order[snd[order] == k][:cap] for k in range(S)])
    assert len(q) == len(keep) and q.senders == S
    b, s = q.consume((1 << 63) - 1, keys)
    idx = b.value[:, :4].copy().view(np.uint32).ravel()
    assert idx.tolist() == keep.tolist()
    assert s.tolist() == snd[keep].tolist()
    q.close()


@pytest.mark.gpu
def test_extreme_keys_and_empty_inputs(verifier):
    """int64-extreme heights / rounds (InvalidRound = -1, negative and maximal
    values) order exactly like the restatement; empty batches, batches with no
    insertable message, and consume/drop on an empty queue are no-ops."""
    import torch
    from hyperdrive_amd.device import DeviceBatch
    from hyperdrive_amd.mq import MessageQueue
    rng = np.random.default_rng(77)
    ext = np.array([-(1 << 63), -(1 << 62), -2, -1, 0, 1, 2, (1 << 62), (1 << 63) - 1], dtype=np.int64)
    keys = _senders(rng, 4)
    q = MessageQueue(verifier, 5)
    o = OracleMQ(5)
    ids = {}
    b, s = q.consume(0, keys)
    assert len(b) == 0 and len(s) == 0 and len(q) == 0
    q.drop_below(1 << 40)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    empty = DeviceBatch(0, t(np.zeros(0, np.uint8)), t(np.zeros(0, np.int64)), t(np.zeros(0, np.int64)),
                        t(np.zeros(0, np.int64)), t(np.zeros((0, 32), np.uint8)), t(np.zeros((0, 32), np.uint8)),
                        t(np.zeros((0, 65), np.uint8)))
    q.insert_device(empty, t(np.zeros(0, np.uint8)))
    for step in range(6):
        n = 400
        h = rng.choice(ext, n)
        r = rng.choice(ext, n)
        typ = rng.integers(1, 4, n).astype(np.uint8)
        val = rng.integers(0, 256, (n, 32), dtype=np.uint8)
        snd = rng.integers(-1, 4, n).astype(np.int32)
        if step == 3:
            snd[:] = -1                                    # nothing insertable
        frm = keys[np.maximum(snd, 0)]
        db = DeviceBatch(n, t(typ), t(h), t(r), t(np.full(n, -1, np.int64)), t(val), t(frm),
                         t(np.zeros((n, 65), np.uint8)))
        q.insert_device(db, t((snd >= 0).astype(np.uint8)))
        for i in range(n):
            if snd[i] >= 0:
                o.insert(frm[i].tobytes(), (int(h[i]), int(r[i]), int(typ[i]), -1, val[i].tobytes(),
                                            frm[i].tobytes(), bytes(65)))
        assert len(q) == len(o)
    hh = int(ext[4])
    b, s = q.consume(hh, keys)
    n_o, want = o.consume(hh)
    _check_consumed(b, s, want, ids)
    q.drop_below(int(ext[7]))
    o.drop_below(int(ext[7]))
    b, s = q.consume((1 << 63) - 1, keys)
    n_o, want = o.consume((1 << 63) - 1)
    _check_consumed(b, s, want, ids)
    assert len(q) == 0
    q.close()
