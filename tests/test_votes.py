"""Incremental vote logs / count table (include/hd_votes.h)
against the restatement of process.go's logs and O(n) counting loops
(oracle/votes_oracle.py).  Host code only: runs without a GPU.

- random insert / trace / reset sequences: every status, logged value, count,
  log length and trace length equals the restatement's after every step;
- batch insert == sequential inserts, with double_of naming the logged vote;
- the process_test-style threshold scenarios (tests/tally_cases.py) give the
  same predicates through quorum.decide_votes as through the restatement;
- C3-sized (1000 signers x 64 rounds) logs, resets reuse memory correctly;
- argument errors are HD_EINVAL, verdicts gate insertion, proposes are not votes;
- with f set, every insert's quorum-crossing events (L47's == 2f+1 on the
  precommit log, process.go:658; L34; L55) equal the restatement's, and a
  round holding more than 2f+1 precommits reports exactly one crossing."""
import random

import numpy as np
import pytest

import votes_oracle as VO
from tally_cases import scenarios
from util import to_np


@pytest.fixture(scope="module")
def V():
    from hyperdrive_amd import votes
    return votes


def _sig(i):
    return (i * 0x9E3779B1 & 0xFFFFFFFF).to_bytes(4, "big") * 8


def _val(i):
    return bytes(32) if i == 0 else bytes([i]) * 32


def _compare_all(v, o, rounds, signers, values):
    for t in (VO.PREVOTE, VO.PRECOMMIT):
        for r in rounds:
            assert v.len(t, r) == o.len(t, r)
            for x in values:
                assert v.count(t, r, x) == o.count(t, r, x), (t, r)
            for s in signers:
                assert v.get(t, r, s) == o.get(t, r, s)
    for r in rounds:
        assert v.trace_len(r) == o.trace_len(r)


@pytest.mark.parametrize("seed", range(4))
def test_random_sequences_match_restatement(V, seed):
    rng = random.Random(seed)
    signers = [_sig(i) for i in range(12)]
    values = [_val(i) for i in range(4)]
    rounds = list(range(-1, 5))
    f = 1 + seed
    v = V.VoteLog(7)
    v.set_f(f)
    o = VO.VoteLogs(7, f)
    for step in range(600):
        op = rng.random()
        if op < 0.85:
            t = rng.choice([VO.PREVOTE, VO.PRECOMMIT])
            h = rng.choice([7, 7, 7, 7, 8, 6]) + (o.height - 7)
            args = (t, h, rng.choice(rounds), rng.choice(values), rng.choice(signers))
            assert v.insert(*args) == o.insert(*args)
            assert v.last_events == o.last_events
        elif op < 0.97:
            r, s = rng.choice(rounds), rng.choice(signers)
            v.trace_propose(r, s)
            o.trace_propose(r, s)
            assert v.last_events == o.last_events
        else:
            h = o.height + rng.choice([0, 1])
            v.reset(h)
            o.reset(h)
            assert v.height == h
        if step % 50 == 0:
            _compare_all(v, o, rounds, signers, values)
    _compare_all(v, o, rounds, signers, values)
    v.close()


def test_batch_insert_equals_sequential(V):
    from hyperdrive_amd.verify import Batch
    rng = np.random.default_rng(5)
    n = 4000
    typ = rng.integers(1, 5, n).astype(np.uint8)               # 1 propose, 4 timeout: not votes
    h = rng.choice([3, 3, 3, 4], n).astype(np.int64)
    r = rng.integers(0, 6, n).astype(np.int64)
    val = np.zeros((n, 32), np.uint8)
    val[:, 0] = rng.integers(0, 3, n)
    frm = np.zeros((n, 32), np.uint8)
    frm[:, :2] = rng.integers(0, 256, (n, 2))
    frm[:, 1] %= 2                                               # 512 signers
    verdict = np.where(rng.random(n) < 0.1, 5, 0).astype(np.uint8)
    b = Batch(typ, h, r, None, val, frm, np.zeros((n, 65), np.uint8))
    v = V.VoteLog(3)
    v.set_f(40)
    status, double_of = v.insert_batch(b, verdict)
    events = v.last_events.copy()
    o = VO.VoteLogs(3, 40)
    first = {}
    for i in range(n):
        if verdict[i] != 0:
            assert status[i] == V.SKIPPED
            continue
        if typ[i] not in (2, 3):
            assert status[i] == V.NOT_VOTE
            continue
        key = (int(typ[i]), int(r[i]), frm[i].tobytes())
        st, prior = o.insert(int(typ[i]), int(h[i]), int(r[i]), val[i].tobytes(), frm[i].tobytes())
        assert status[i] == st, i
        assert events[i] == o.last_events, i
        if st == VO.INSERTED:
            first[key] = i
        if st == VO.DOUBLE:
            assert double_of[i] == first[key] and val[first[key]].tobytes() == prior
        else:
            assert double_of[i] == V.NO_INDEX
    # a second batch: doubles against the first batch's votes have no index in this call
    s2, d2 = v.insert_batch(b, verdict)
    ok = (verdict == 0) & np.isin(typ, [2, 3]) & (h == 3)
    assert set(s2[ok].tolist()) <= {V.DUPLICATE, V.DOUBLE}
    assert (d2 == V.NO_INDEX).all()
    assert int((events != 0).sum()) > 0
    _compare_all(v, o, range(6), [frm[i].tobytes() for i in range(0, n, 97)], [_val(0), _val(1), _val(2)])


@pytest.mark.parametrize("sc", scenarios(), ids=lambda s: s.name)
def test_scenarios_through_vote_log(V, oracle, sc):
    """process_test-style thresholds (tests/tally_cases.py) through the
    incremental table: same predicates as the restatement's tally."""
    from hyperdrive_amd import quorum
    b = to_np(sc.b)
    t = oracle.tally(sc.b, sc.verdicts())
    for h, r, pvalue, pvalid, want in sc.expect:
        v = V.VoteLog(h)
        v.insert_batch(b)
        got = quorum.decide_votes(v, r, sc.f, pvalue, pvalid)
        ref = oracle.decide_round(t, h, r, sc.f, pvalue, pvalid)
        assert got == ref
        for k, x in want.items():
            assert got[k] == x, (sc.name, k)
        v.close()


def test_c3_sized_logs_and_reset(V):
    """C3 shape: 1000 signers, 64 rounds, one prevote + one
    precommit each, values 90% canonical / 5% nil / 5% other; then a reset
    to the next height and a smaller second height in reused memory."""
    from hyperdrive_amd.verify import Batch
    rng = np.random.default_rng(7)
    S, R = 1000, 64
    n = 2 * S * R
    i = np.arange(n)
    r = (i // (2 * S)).astype(np.int64)
    typ = (2 + i % 2).astype(np.uint8)
    signer = (i // 2) % S
    frm = np.zeros((n, 32), np.uint8)
    frm[:, :4] = signer.astype(np.uint32).view(np.uint8).reshape(n, 4)
    frm[:, 31] = 0xA5
    u = rng.random(n)
    val = np.zeros((n, 32), np.uint8)
    val[:, 0] = np.where(u < 0.9, 1, np.where(u < 0.95, 0, 2))
    val[:, 1] = np.where(u >= 0.95, rng.integers(0, 256, n), 0)
    val[:, 8:16] = r.astype(np.int64).view(np.uint8).reshape(n, 8) * (u < 0.9)[:, None]
    b = Batch(typ, np.ones(n, np.int64), r, None, val, frm, np.zeros((n, 65), np.uint8))
    v = V.VoteLog(1)
    status, _ = v.insert_batch(b)
    assert (status == V.INSERTED).all()
    for rr in (0, 17, 63):
        for t in (2, 3):
            sel = (r == rr) & (typ == t)
            assert v.len(t, rr) == S
            for x in {val[k].tobytes() for k in np.flatnonzero(sel)[:50]}:
                assert v.count(t, rr, x) == int((val[sel] == np.frombuffer(x, np.uint8)).all(1).sum())
        assert v.trace_len(rr) == S
    v.reset(2)
    assert v.len(2, 0) == 0 and v.trace_len(0) == 0 and v.count(2, 0, _val(0)) == 0
    b2 = Batch(typ[:500], np.full(500, 2, np.int64), r[:500], None, val[:500], frm[:500], np.zeros((500, 65), np.uint8))
    st, _ = v.insert_batch(b2)
    assert (st == V.INSERTED).all() and v.len(2, 0) == 250 and v.len(3, 0) == 250 and v.trace_len(0) == 250
    v.close()


def test_errors_and_edges(V):
    from hyperdrive_amd import _lib
    from hyperdrive_amd.verify import Batch
    v = V.VoteLog(0)
    with pytest.raises(_lib.HDError):
        v.count(1, 0, _val(0))                 # a propose is not a vote log
    with pytest.raises(_lib.HDError):
        v.insert(4, 0, 0, _val(0), _sig(1))
    with pytest.raises(ValueError):
        v.insert(2, 0, 0, b"short", _sig(1))
    e = Batch(np.zeros(0, np.uint8), np.zeros(0, np.int64), np.zeros(0, np.int64), None,
              np.zeros((0, 32), np.uint8), np.zeros((0, 32), np.uint8), np.zeros((0, 65), np.uint8))
    st, d = v.insert_batch(e)
    assert len(st) == 0 and len(d) == 0
    assert v.count(2, 99, _val(0)) == 0 and v.len(3, -5) == 0 and v.trace_len(1 << 40) == 0
    # extreme rounds / heights are plain keys
    assert v.insert(2, 0, (1 << 63) - 1, _val(1), _sig(1)) == (V.INSERTED, None)
    assert v.insert(2, 0, -(1 << 63), _val(1), _sig(1)) == (V.INSERTED, None)
    assert v.insert(2, 0, (1 << 63) - 1, _val(2), _sig(1)) == (V.DOUBLE, _val(1))
    assert v.insert(2, 1, 0, _val(1), _sig(1)) == (V.WRONG_HEIGHT, None)
    v.close()


def test_precommit_crossing_reported_once(V):
    """L47 (process.go:658) is len(PrecommitLogs[r]) == 2f+1: over 2f+3
    precommits of one round (duplicates and a double vote among them) exactly
    the insert of the (2f+1)-th distinct signer crosses; the prevote log and
    the trace report their own crossings; a round entered afterwards holds
    2f+3 > 2f+1 logs, so StartRound's equality (quorum 'timeout_precommit_exact')
    is false while 'timeout_precommit_reached' is true."""
    from hyperdrive_amd import quorum
    for f in (1, 5, 33):
        v = V.VoteLog(9)
        v.set_f(f)
        o = VO.VoteLogs(9, f)
        crossed = []
        for k in range(2 * f + 3):
            for frm in (_sig(k), _sig(k)):                     # an identical duplicate each time
                st, _ = v.insert(VO.PRECOMMIT, 9, 2, _val(1), frm)
                o.insert(VO.PRECOMMIT, 9, 2, _val(1), frm)
                assert v.last_events == o.last_events
                if v.last_events & V.EV_PRECOMMIT_2F1:
                    crossed.append(k)
        st, _ = v.insert(VO.PRECOMMIT, 9, 2, _val(2), _sig(0))   # double vote: no event
        assert st == V.DOUBLE and v.last_events == 0
        assert crossed == [2 * f]
        d = quorum.decide_votes(v, 2, f)
        assert d["timeout_precommit_reached"] and not d["timeout_precommit_exact"]
        v.reset(10)
        for k in range(2 * f + 1):
            v.insert(VO.PRECOMMIT, 10, 0, _val(1), _sig(k))
        d = quorum.decide_votes(v, 0, f)
        assert d["timeout_precommit_reached"] and d["timeout_precommit_exact"]
        v.close()
