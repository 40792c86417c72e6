"""Tally scenarios restating the threshold behaviour the reference's
process_test.go pins (2f vs 2f+1, f vs f+1, first-wins, mixed values, caught
double votes).  Each returns (batch lists, verdicts, expectations)."""
from __future__ import annotations

import random

import hd_pyoracle as O

PV, PC = O.PREVOTE, O.PRECOMMIT


def _sig(i: int) -> bytes:
    return O.sha256(b"signer" + i.to_bytes(4, "big"))


class Scenario:
    def __init__(self, name, f):
        self.name = name
        self.f = f
        self.b = O.Batch()
        self.expect = []  # (h, r, propose_value, propose_valid, {pred: bool})

    def vote(self, t, h, r, signer, value):
        self.b.append(t, h, r, -1, value, _sig(signer), bytes(65))

    def verdicts(self):
        return [O.VALID] * len(self.b)


def scenarios(seed: int = 1):
    rng = random.Random(seed)
    out = []
    for f in [5, 17, 33, 49]:
        v = O.canonical_value(1, 0)
        # 1. 2f distinct prevotes for v -> nothing; 2f+1 -> timeout/precommit (process_test.go:1590-1866, 1879-2220)
        s = Scenario(f"prevotes_2f_f{f}", f)
        for k in range(2 * f):
            s.vote(PV, 1, 0, k, v)
        s.expect.append((1, 0, v, True, {"timeout_prevote": False, "precommit_value": False}))
        out.append(s)
        s = Scenario(f"prevotes_2f1_f{f}", f)
        for k in range(2 * f + 1):
            s.vote(PV, 1, 0, k, v)
        s.expect.append((1, 0, v, True, {"timeout_prevote": True, "precommit_value": True, "commit": False}))
        out.append(s)
        # 2. duplicates of one signer never reach the threshold (first-wins, process.go:834-845)
        s = Scenario(f"dups_f{f}", f)
        for k in range(2 * f):
            s.vote(PV, 1, 0, k, v)
        for _ in range(5):
            s.vote(PV, 1, 0, 0, v)                     # identical duplicate: dropped, not caught
        s.vote(PV, 1, 0, 1, O.canonical_value(9, 9))  # double vote: caught, not counted
        s.expect.append((1, 0, v, True, {"timeout_prevote": False, "precommit_value": False}))
        out.append(s)
        # 3. nil prevotes (process_test.go:2222-2425)
        s = Scenario(f"nil_f{f}", f)
        for k in range(2 * f + 1):
            s.vote(PV, 2, 3, k, O.NIL_VALUE)
        s.expect.append((2, 3, v, True, {"precommit_nil": True, "precommit_value": False, "timeout_prevote": True}))
        out.append(s)
        # 4. precommits: 2f+1 for the propose value -> commit; mixed values -> no commit (2639-3277, 3009-3070)
        s = Scenario(f"commit_f{f}", f)
        for k in range(2 * f + 1):
            s.vote(PC, 5, 1, k, v)
        s.expect.append((5, 1, v, True, {"commit": True, "timeout_precommit_reached": True}))
        s.expect.append((5, 1, v, False, {"commit": False}))   # invalid propose never commits (687-694)
        out.append(s)
        # a round holding more than 2f+1 precommits: StartRound's L47 equality
        # (process.go:310, 658) does not fire, though the log passed 2f+1
        s = Scenario(f"precommits_over_2f1_f{f}", f)
        for k in range(2 * f + 3):
            s.vote(PC, 6, 2, k, v)
        s.expect.append((6, 2, v, True, {"timeout_precommit_reached": True, "timeout_precommit_exact": False}))
        out.append(s)
        s = Scenario(f"precommits_exact_2f1_f{f}", f)
        for k in range(2 * f + 1):
            s.vote(PC, 6, 2, k, O.canonical_value(6, 7) if k % 3 == 0 else v)
        s.expect.append((6, 2, v, True, {"timeout_precommit_reached": True, "timeout_precommit_exact": True,
                                         "commit": False}))
        out.append(s)
        s = Scenario(f"mixed_f{f}", f)
        for k in range(2 * f + 1):
            s.vote(PC, 5, 1, k, v if k % 2 == 0 else O.canonical_value(5, 99))
        s.expect.append((5, 1, v, True, {"commit": False, "timeout_precommit_reached": True}))
        out.append(s)
        # 5. f vs f+1 unique signers across prevote and precommit (3279-3802)
        s = Scenario(f"skip_f{f}", f)
        for k in range(f):
            s.vote(PV if k % 2 else PC, 7, 4, k, v)
        s.vote(PC, 7, 4, 0, v)    # same signer again in the other log: not a new signatory
        s.expect.append((7, 4, v, True, {"skip": False}))
        out.append(s)
        s = Scenario(f"skip1_f{f}", f)
        for k in range(f + 1):
            s.vote(PV if k % 2 else PC, 7, 4, k, v)
        s.expect.append((7, 4, v, True, {"skip": True}))
        out.append(s)
        # 6. votes at other heights / rounds never leak into (h, r)
        s = Scenario(f"isolation_f{f}", f)
        for k in range(2 * f + 1):
            s.vote(PV, 1 + (k % 2), k % 3, k, v)
        s.expect.append((1, 0, v, True, {"timeout_prevote": False}))
        out.append(s)
    # 7. a random shuffle of everything, with interleaved signers
    s = Scenario("random_mix", 20)
    vals = [O.canonical_value(1, r) for r in range(4)] + [O.NIL_VALUE]
    for _ in range(3000):
        s.vote(rng.choice([PV, PC]), rng.randrange(1, 4), rng.randrange(0, 4), rng.randrange(0, 70),
               rng.choice(vals))
    out.append(s)
    return out
