"""Bulk MessageQueue (include/hd_mq.h) against the one-message-at-a-time
restatement of mq/mq.go (oracle/mq_oracle.py).

CPU: the restatement reproduces the reference's own mq_test.go behaviours --
max capacity 1 (mq_test.go:642-714), excess dropped (716-793), ordering by
height and round (334-608), drop below height (611-639), procsAllowed at
consume (119-331).
GPU: random insert / consume / drop sequences give exactly the restatement's
consumed messages (all fields, order included) for capacities 1, 3, 25 and
1000; a 1M-message batch from 100 senders keeps every sender's 1000 smallest
(height, round, arrival) messages."""
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


# ---------------------------------------------------------------- GPU
@pytest.fixture(scope="module")
def verifier(gpu):
    v = gpu.Verifier(0)
    yield v
    v.close()


def _batch(rng, n, S, hmax, rmax, neg_pct=10):
    import torch
    from hyperdrive_amd.device import DeviceBatch
    typ = rng.integers(1, 4, n).astype(np.uint8)
    h = rng.integers(0, hmax, n).astype(np.int64)
    r = rng.integers(0, rmax, n).astype(np.int64)
    vr = rng.integers(-1, 3, n).astype(np.int64)
    value = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    frm = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    sig = rng.integers(0, 256, (n, 65), dtype=np.uint8)
    snd = rng.integers(0, S, n).astype(np.int32)
    snd[rng.random(n) < neg_pct / 100] = -1
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    db = DeviceBatch(n, t(typ), t(h), t(r), t(vr), t(value), t(frm), t(sig))
    host = [(int(h[i]), int(r[i]), int(typ[i]), int(vr[i]), value[i].tobytes(), frm[i].tobytes(), sig[i].tobytes())
            for i in range(n)]
    return db, t(snd), host, snd


def _as_tuples(b, snd):
    return [(int(snd[k]), (int(b.height[k]), int(b.round[k]), int(b.type[k]), int(b.valid_round[k]),
                           b.value[k].tobytes(), b.frm[k].tobytes(), b.sig[k].tobytes())) for k in range(len(b))]


@pytest.mark.gpu
@pytest.mark.parametrize("cap", [1, 3, 25, 1000])
def test_random_sequences_match_oracle(verifier, cap):
    from hyperdrive_amd.mq import MessageQueue
    rng = np.random.default_rng(cap)
    q = MessageQueue(verifier, cap)
    o = OracleMQ(cap)
    for step in range(12):
        db, d_snd, host, snd = _batch(rng, int(rng.integers(1, 3000)), 7, 6, 4)
        q.insert_device(db, d_snd)
        for i, m in enumerate(host):
            if snd[i] >= 0:
                o.insert(int(snd[i]), m)
        assert len(q) == len(o)
        op = step % 3
        if op == 1:
            hh = int(rng.integers(0, 6))
            b, s = q.consume(hh)
            n, want = o.consume(hh)
            assert _as_tuples(b, s) == want and len(b) == n
        elif op == 2:
            hh = int(rng.integers(0, 6))
            q.drop_below(hh)
            o.drop_below(hh)
    b, s = q.consume(10 ** 9)
    n, want = o.consume(10 ** 9)
    assert _as_tuples(b, s) == want
    q.close()


@pytest.mark.gpu
def test_capacity_one_on_gpu(verifier):
    """mq_test.go:642-714 through the GPU queue."""
    import torch
    from hyperdrive_amd.device import DeviceBatch
    from hyperdrive_amd.mq import MessageQueue

    def one(h, r, sender, tag):
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
        val = np.zeros((1, 32), np.uint8)
        val[0, 0] = tag
        db = DeviceBatch(1, t(np.array([1], np.uint8)), t(np.array([h], np.int64)), t(np.array([r], np.int64)),
                         t(np.array([-1], np.int64)), t(val), t(np.zeros((1, 32), np.uint8)),
                         t(np.zeros((1, 65), np.uint8)))
        return db, t(np.array([sender], np.int32))

    q = MessageQueue(verifier, 1)
    q.insert_device(*one(1, 1, 0, 1))
    q.insert_device(*one(1, 2, 1, 2))
    b, s = q.consume(1)
    assert len(b) == 2
    q.insert_device(*one(1, 1, 0, 1))
    q.insert_device(*one(1, 2, 0, 3))
    b, s = q.consume(1)
    assert len(b) == 1 and b.value[0, 0] == 1
    q.insert_device(*one(1, 1, 0, 1))
    q.insert_device(*one(1, 0, 0, 4))
    b, s = q.consume(1)
    assert len(b) == 1 and b.value[0, 0] == 4
    q.close()


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
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    tag = np.zeros((n, 32), np.uint8)
    tag[:, :4] = np.arange(n, dtype=np.uint32).view(np.uint8).reshape(n, 4)
    db = DeviceBatch(n, t(np.full(n, 2, np.uint8)), t(h), t(r), t(np.full(n, -1, np.int64)), t(tag),
                     t(np.zeros((n, 32), np.uint8)), t(np.zeros((n, 65), np.uint8)))
    q = MessageQueue(verifier, 1000)
    q.insert_device(db, t(snd))
    assert len(q) == S * 1000
    b, s = q.consume(10 ** 9)
    idx = b.value[:, :4].copy().view(np.uint32).ravel()
    order = np.lexsort((np.arange(n), r, h, snd))           # sender, h, r, arrival
    keep = np.concatenate([order[snd[order] == k][:1000] for k in range(S)])
    assert idx.tolist() == keep.tolist()
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
    q = MessageQueue(verifier, 5)
    o = OracleMQ(5)
    b, s = q.consume(0)
    assert len(b) == 0 and len(s) == 0 and len(q) == 0
    q.drop_below(1 << 40)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    empty = DeviceBatch(0, t(np.zeros(0, np.uint8)), t(np.zeros(0, np.int64)), t(np.zeros(0, np.int64)),
                        t(np.zeros(0, np.int64)), t(np.zeros((0, 32), np.uint8)), t(np.zeros((0, 32), np.uint8)),
                        t(np.zeros((0, 65), np.uint8)))
    q.insert_device(empty, t(np.zeros(0, np.int32)))
    for step in range(6):
        n = 400
        h = rng.choice(ext, n)
        r = rng.choice(ext, n)
        typ = rng.integers(1, 4, n).astype(np.uint8)
        val = rng.integers(0, 256, (n, 32), dtype=np.uint8)
        snd = rng.integers(-1, 4, n).astype(np.int32)
        if step == 3:
            snd[:] = -1                                    # nothing insertable
        db = DeviceBatch(n, t(typ), t(h), t(r), t(np.full(n, -1, np.int64)), t(val), t(np.zeros((n, 32), np.uint8)),
                         t(np.zeros((n, 65), np.uint8)))
        q.insert_device(db, t(snd))
        for i in range(n):
            if snd[i] >= 0:
                o.insert(int(snd[i]), (int(h[i]), int(r[i]), int(typ[i]), -1, val[i].tobytes(), bytes(32),
                                       bytes(65)))
        assert len(q) == len(o)
    hh = int(ext[4])
    b, s = q.consume(hh)
    n_o, want = o.consume(hh)
    assert _as_tuples(b, s) == want
    q.drop_below(int(ext[7]))
    o.drop_below(int(ext[7]))
    b, s = q.consume((1 << 63) - 1)
    n_o, want = o.consume((1 << 63) - 1)
    assert _as_tuples(b, s) == want and len(q) == 0
    q.close()
