"""CPU restatement of the vote logs a Process keeps for its current height,
and of the O(n) counting loops its rules run over them.

TEST INFRASTRUCTURE ONLY: the checker of include/hd_votes.h in tests/; the
product never imports it.

  state         process/state.go:44-57     PrevoteLogs / PrecommitLogs
                                           map[Round]map[Signatory]vote,
                                           TraceLogs map[Round]map[Signatory]bool
  insert vote   process.go:823-855, 860-892  h == CurrentHeight; first wins
                                           per (round, From); an Equal vote is
                                           dropped silently, a different one is
                                           a double vote (Catcher); an accepted
                                           vote adds From to TraceLogs[round]
  valid propose process.go:810-815         TraceLogs[round][From] = true
  counts        process.go:486-491 (L28), 574-579 (L36), 626-631 (L44),
                696-701 (L49): a loop over the round's log comparing values
  lengths       process.go:534 (L34), 658 (L47), 751 (L55)
  crossings     with f set: the insert that makes len(PrecommitLogs[r]) ==
                2f+1 (L47's equality, tried after every precommit insert,
                process.go:268), len(PrevoteLogs[r]) == 2f+1 (L34) or
                |TraceLogs[r]| == f+1 (L55) reports it (last_events)
  reset         process.go:718-724         every log emptied at a new height

A vote is (value: bytes32); Prevote.Equal compares height, round, value and
from (message.go), of which only value can differ between two votes logged
under the same (round, From) of one height.
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

PREVOTE, PRECOMMIT = 2, 3
INSERTED, WRONG_HEIGHT, DUPLICATE, DOUBLE = 0, 1, 2, 3
EV_PREVOTE_2F1, EV_PRECOMMIT_2F1, EV_TRACE_F1 = 1, 2, 4


class VoteLogs:
    def __init__(self, height: int = 0, f: Optional[int] = None):
        self.f = f
        self.last_events = 0
        self.reset(height)

    def reset(self, height: int) -> None:
        self.height = height
        self.logs: Dict[int, Dict[int, Dict[bytes, bytes]]] = {PREVOTE: {}, PRECOMMIT: {}}
        self.trace: Dict[int, Dict[bytes, bool]] = {}

    def insert(self, mtype: int, height: int, round_: int, value: bytes, frm: bytes) -> Tuple[int, Optional[bytes]]:
        self.last_events = 0
        if height != self.height:
            return WRONG_HEIGHT, None
        log = self.logs[mtype].setdefault(round_, {})
        if frm in log:
            prior = log[frm]
            return (DUPLICATE, None) if prior == value else (DOUBLE, prior)
        log[frm] = value
        tr = self.trace.setdefault(round_, {})
        fresh = frm not in tr
        tr[frm] = True
        if self.f is not None:
            if len(log) == 2 * self.f + 1:                    # process.go:534 / 658
                self.last_events |= EV_PREVOTE_2F1 if mtype == PREVOTE else EV_PRECOMMIT_2F1
            if fresh and len(tr) == self.f + 1:               # process.go:751
                self.last_events |= EV_TRACE_F1
        return INSERTED, None

    def trace_propose(self, round_: int, frm: bytes) -> None:
        tr = self.trace.setdefault(round_, {})
        fresh = frm not in tr
        tr[frm] = True
        self.last_events = EV_TRACE_F1 if (self.f is not None and fresh and len(tr) == self.f + 1) else 0

    def count(self, mtype: int, round_: int, value: bytes) -> int:
        n = 0
        for v in self.logs[mtype].get(round_, {}).values():     # the reference's O(n) loop
            if v == value:
                n += 1
        return n

    def len(self, mtype: int, round_: int) -> int:
        return len(self.logs[mtype].get(round_, {}))

    def trace_len(self, round_: int) -> int:
        return len(self.trace.get(round_, {}))

    def get(self, mtype: int, round_: int, frm: bytes) -> Optional[bytes]:
        return self.logs[mtype].get(round_, {}).get(frm)
