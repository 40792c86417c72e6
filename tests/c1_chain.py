"""The C1 plumbing config -- BASELINE configs[0], "4 replicas (f=1), 100
heights" -- as one replica's view of the message stream: the messages every
replica of an honest n = 4 network broadcasts over 100 heights (one propose by
the round-robin proposer, 4 prevotes and 4 precommits per height), delivered in
arrival chunks with heights out of order, plus re-sent duplicates, a double
vote, forged signatures, an outsider's votes and stale heights.

Reference shape: replica/replica_test.go:378-430 (n replicas over an
in-memory network until every replica commits the same values) with
SURVEY F10's parameters (f = 1, n = 4, 100 heights).  One replica's chain is
what this file drives, twice over the same arrival stream:

  chain="oracle"  (test infrastructure: CPU restatements) C oracle verdicts
                  (libsecp256k1 semantics) -> filterHeight (replica.go:247-249)
                  -> mq_oracle insert of authenticated messages (mq.go:103-143)
                  -> mq_oracle.consume(h, procsAllowed) (mq.go:36-66)
                  -> votes_oracle logs (process.go:823-892)
  chain="gpu"     hyperdrive_amd.Ingress: wire bytes -> unmarshal -> verify ->
                  filterHeight -> mq insert -> consume -> vote logs (HIP + host)

After each chunk the replica flushes until it cannot commit (replica.go:
251-264 loops Consume; a commit moves the Process to h + 1, process.go:
703-728): proposes go to the CPU's insertPropose (the scheduled proposer
(h + r) % n, scheduler.go:31-53; a valid propose joins TraceLogs,
process.go:810-815) and the quorum predicates (hyperdrive_amd.quorum,
process.go L28-L55 with f = 1: 2f+1 = 3, f+1 = 2) decide.  Every flush is
recorded; both chains must produce the same records.
"""
from __future__ import annotations

import numpy as np

PROPOSE, PREVOTE, PRECOMMIT = 1, 2, 3
N_SIGNERS, HEIGHTS, CHUNK = 4, 100, 10


def make_stream(O):
    """The arrival stream (numpy arrays, arrival order) and the admitted set.
    O = oracle/hd_pyoracle (signing with RFC6979, SEC1-compressed signatories)."""
    rng = np.random.default_rng(0xC1)
    sks = [O.signer_sk(i) for i in range(N_SIGNERS + 1)]        # signer 4 is an outsider
    sigs = [O.signatory_of_pub(O.pubkey_of(sk), True) for sk in sks]
    msgs = []   # (chunk, type, h, r, vr, value, signer, sign_h)

    def add(t, h, value, s, chunk=None, sign_h=None, vr=-1):
        if chunk is None:
            u = rng.random()
            delay = 0 if u < 0.7 else (int(rng.integers(3, 13)) if u < 0.9 else -int(rng.integers(1, 9)))
            chunk = min(max((h - 1 + delay) // CHUNK, 0), HEIGHTS // CHUNK - 1)
            if h <= 50:
                chunk = min(chunk, 4)      # the replica stands at height 50 after chunk 4 (the 2f boundary)
        msgs.append((chunk, t, h, 0, vr, value, s, h if sign_h is None else sign_h))

    nil = bytes(32)
    for h in range(1, HEIGHTS + 1):
        V = O.canonical_value(h, 0)
        add(PROPOSE, h, V, h % N_SIGNERS)                               # (h + r) % n, r = 0
        for s in range(N_SIGNERS):
            add(PREVOTE, h, nil if (h % 10 == 0 and s == 3) else V, s)
        pcs = [0, 1, 2, 3]
        if h % 7 == 0:
            pcs = [0, 1, 2]                                             # one replica silent: exactly 2f+1
        if h == 50:
            pcs = [0, 1]                                                # 2f on time ...
            add(PRECOMMIT, h, V, 2, chunk=(h - 1) // CHUNK + 1)         # ... the third a chunk later
        for s in pcs:
            add(PRECOMMIT, h, V, s, chunk=(h - 1) // CHUNK if h == 50 else None)
        if h % 5 == 0:
            add(PREVOTE, h, V, 0)                                       # re-sent: identical duplicate
        if h % 13 == 0 and h % 7 != 0:
            add(PRECOMMIT, h, O.random_value(h), 1)                     # double vote (3 honest remain)
        if h % 11 == 0:
            add(PREVOTE, h, V, 2, sign_h=h + 1000)                      # signature over another digest
        if h % 9 == 0:
            add(PREVOTE, h, V, 4)                                       # authenticated, never admitted
        if h > 5 and h % 6 == 0:
            add(PREVOTE, h - 5, O.canonical_value(h - 5, 0), 1, chunk=(h - 1) // CHUNK)   # stale height
    # arrival: by chunk; inside a chunk the propose, prevote and precommit
    # wire buffers in that order, each shuffled (heights out of order)
    order = []
    for c in range(HEIGHTS // CHUNK):
        for t in (PROPOSE, PREVOTE, PRECOMMIT):
            idx = [k for k, m in enumerate(msgs) if m[0] == c and m[1] == t]
            rng.shuffle(idx)
            order += idx
    n = len(order)
    out = {k: np.zeros(n, dt) for k, dt in (("chunk", np.int32), ("type", np.uint8), ("height", np.int64),
                                             ("round", np.int64), ("valid_round", np.int64))}
    out["value"] = np.zeros((n, 32), np.uint8)
    out["frm"] = np.zeros((n, 32), np.uint8)
    out["sig"] = np.zeros((n, 65), np.uint8)
    for j, k in enumerate(order):
        c, t, h, r, vr, value, s, sh = msgs[k]
        out["chunk"][j], out["type"][j], out["height"][j], out["round"][j], out["valid_round"][j] = c, t, h, r, vr
        out["value"][j] = np.frombuffer(value, np.uint8)
        out["frm"][j] = np.frombuffer(sigs[s], np.uint8)
        out["sig"][j] = np.frombuffer(O.sign(sks[s], O.message_digest(t, sh, r, vr, value)), np.uint8)
    out["admitted"] = np.array([np.frombuffer(x, np.uint8) for x in sigs[:N_SIGNERS]])
    return out


def replica_view(z, k: int, replicas: int = 4):
    """Replica k's arrival of the same network stream (BASELINE configs[0]: 4
    replicas, f = 1, 100 heights; replica/replica_test.go:378-423 runs n
    replicas over one in-memory network): replica 0 sees the committed
    order; replica k > 0 sees the same signed messages chunked with its own
    random delays (-2 .. +6 chunks) and shuffled inside each chunk's
    propose / prevote / precommit buffers."""
    if k == 0:
        return z
    rng = np.random.default_rng(0xC1 + 17 * k)
    n = len(z["type"])
    h = z["height"].astype(np.int64)
    chunk = np.clip((h - 1) // CHUNK + rng.integers(-2, 7, n), 0, HEIGHTS // CHUNK - 1)
    order = np.lexsort((rng.random(n), z["type"], chunk))
    out = {key: (val if key == "admitted" else val[order]) for key, val in z.items()}
    out["chunk"] = chunk[order].astype(np.int32)
    return out


def _batch(z, idx):
    from hyperdrive_amd.verify import Batch
    return Batch(z["type"][idx], z["height"][idx], z["round"][idx], z["valid_round"][idx], z["value"][idx],
                 z["frm"][idx], z["sig"][idx])


class _Replica:
    """The CPU side both chains share: insertPropose for delivered proposes,
    the predicates, the commit."""

    def __init__(self, admitted):
        self.admitted = [bytes(a) for a in admitted]
        self.f = len(self.admitted) // 3
        self.height = 1
        self.proposal = {}          # height -> value of its valid propose
        self.records = []
        self.commits = []

    def on_flush(self, votes, delivered, statuses, events, proposes):
        from hyperdrive_amd.quorum import decide_votes
        h = self.height
        for (ph, pr, pv, pfrom) in proposes:
            # insertPropose (process.go:758-819): current height, the scheduled
            # proposer (h + r) % n, first wins, a nil value is not valid
            if ph == h and pfrom == self.admitted[(ph + pr) % len(self.admitted)] and h not in self.proposal \
                    and pv != bytes(32):
                self.proposal[h] = pv
                votes.trace_propose(pr, pfrom)
        pv = self.proposal.get(h)
        d = decide_votes(votes, 0, self.f, pv, pv is not None)
        st = np.bincount(np.asarray(statuses, np.int64), minlength=6).tolist() if len(statuses) else [0] * 6
        ev = np.asarray(events, np.uint8)
        self.records.append({"height": h, "delivered": int(delivered), "status": st,
                             "ev_precommit_2f1": int(((ev & 2) != 0).sum()), "ev_prevote_2f1": int(((ev & 1) != 0).sum()),
                             "ev_trace_f1": int(((ev & 4) != 0).sum()), "decision": d})
        if d["commit"]:
            self.commits.append((h, pv.hex()))
            self.height += 1
            return True
        return False


def run_oracle(z, coracle):
    """The chain of CPU restatements (test infrastructure)."""
    import mq_oracle as MQO
    import votes_oracle as VO
    rep = _Replica(z["admitted"])
    mq = MQO.MessageQueue(1000)
    votes = VO.VoteLogs(1, rep.f)
    allowed = set(rep.admitted)
    for c in range(int(z["chunk"].max()) + 1):
        for t in (PROPOSE, PREVOTE, PRECOMMIT):
            idx = np.flatnonzero((z["chunk"] == c) & (z["type"] == t))
            if not len(idx):
                continue
            vd, _ = coracle.verify(_batch(z, idx), z["admitted"], True, threads=4)
            for k, i in enumerate(idx):
                if vd[k] in (0, 6) and z["height"][i] >= rep.height:       # authenticated; filterHeight
                    mq.insert(z["frm"][i].tobytes(), (int(z["height"][i]), int(z["round"][i]), t, i))
        while True:
            n_rm, want = mq.consume(rep.height, allowed=allowed)
            statuses, events, proposes = [], [], []
            for frm, (h, r, t, i) in want:
                if t == PROPOSE:
                    statuses.append(4)           # NOT_VOTE
                    events.append(0)
                    proposes.append((h, r, z["value"][i].tobytes(), frm))
                    continue
                st, _ = votes.insert(t, h, r, z["value"][i].tobytes(), frm)
                statuses.append(st)
                events.append(votes.last_events)
            if not rep.on_flush(votes, len(want), statuses, events, proposes):
                break
            votes.reset(rep.height)
    return rep


def run_gpu(z, verifier):
    """The same stream through hyperdrive_amd.Ingress (wire bytes in)."""
    import torch
    import surge_codec as SC
    from hyperdrive_amd.ingress import Ingress
    verifier.set_signatories(z["admitted"])
    rep = _Replica(z["admitted"])
    ing = Ingress(verifier, height=1, max_capacity=1000)
    assert ing.f == rep.f
    try:
        for c in range(int(z["chunk"].max()) + 1):
            parts = []
            for t in (PROPOSE, PREVOTE, PRECOMMIT):
                idx = np.flatnonzero((z["chunk"] == c) & (z["type"] == t))
                if not len(idx):
                    continue
                vr = z["valid_round"][idx] if t == PROPOSE else None
                buf = SC.marshal_array(t, z["height"][idx], z["round"][idx], vr, z["value"][idx], z["frm"][idx],
                                       z["sig"][idx])
                parts.append((t, torch.frombuffer(bytearray(buf), dtype=torch.uint8).cuda(), len(idx)))
            # even chunks one buffer at a time, odd chunks overlapped (push_wires)
            if c % 2:
                ing.push_wires(parts)
            else:
                for t, buf, n in parts:
                    ing.push_wire(t, buf, n)
            while True:
                res = ing.flush()
                b = res.consumed
                proposes = [(int(b.height[i]), int(b.round[i]), b.value[i].tobytes(), b.frm[i].tobytes())
                            for i in res.proposes]
                ev = res.events if res.events is not None else np.zeros(len(b), np.uint8)
                if not rep.on_flush(ing.votes, len(b), res.vote_status, ev, proposes):
                    break
                ing.advance_height(rep.height)
    finally:
        ing.close()
    return rep
