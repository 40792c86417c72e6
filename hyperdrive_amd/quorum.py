"""Host-side quorum predicates over a batch tally.

The GPU tally (hd_tally) produces, per (height, round), the sizes of the
first-wins vote logs and the per-value counts; these functions apply the exact
comparisons of the reference's rules to them.  The automaton's step / once-flag
gating (process.go's ``CurrentStep`` checks and ``OnceFlag``) is sequential
control flow and stays with the caller.
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

PREVOTE, PRECOMMIT = 2, 3
INVALID_ROUND = -1
NIL_VALUE = bytes(32)


def thresholds(n_signatories: int) -> Tuple[int, int, int]:
    """f = len(signatories) / 3 (integer division, replica/replica.go:54, 138);
    returns (f, 2f+1, f+1)."""
    f = n_signatories // 3
    return f, 2 * f + 1, f + 1


def decide(tally, height: int, round_: int, f: int, propose_value: Optional[bytes] = None,
           propose_valid: bool = False, propose_valid_round: int = INVALID_ROUND,
           propose_signer_new: bool = False) -> Dict[str, bool]:
    """Predicates for one (height, round) given a tally with ``count``,
    ``distinct`` and ``distinct_any`` maps.

    - timeout_prevote   L34 ``len(PrevoteLogs[r]) >= 2f+1``         process.go:534
    - precommit_nil     L44 #prevotes for NilValue >= 2f+1          process.go:626-632
    - timeout_precommit_reached  L47: the log reached 2f+1 at some insert of
      the batch (``>=``: true iff the equality ``len == 2f+1`` held at the
      crossing insert; the per-insert crossing is hd_votes' EV_PRECOMMIT_2F1)
                                                                    process.go:658
    - timeout_precommit_exact  L47 as StartRound evaluates it on entering the
      round: ``len(PrecommitLogs[r]) == 2f+1`` exactly (more than 2f+1
      buffered precommits never fire it)                   process.go:310, 658
    - skip              L55 |TraceLogs[r]| >= f+1 (votes + valid propose signer) process.go:751
    - precommit_value   L36 #prevotes for propose.Value >= 2f+1     process.go:574-582
    - commit            L49 #precommits for propose.Value >= 2f+1   process.go:696-702
    - prevote_validround L28 #prevotes in validRound for propose.Value >= 2f+1  process.go:486-494
    """
    q = 2 * f + 1
    count = tally.count
    pv = lambda v: count.get((height, round_, PREVOTE, v), 0)
    pc = lambda v: count.get((height, round_, PRECOMMIT, v), 0)
    out = {
        "timeout_prevote": tally.distinct.get((height, round_, PREVOTE), 0) >= q,
        "precommit_nil": pv(NIL_VALUE) >= q,
        "timeout_precommit_reached": tally.distinct.get((height, round_, PRECOMMIT), 0) >= q,
        "timeout_precommit_exact": tally.distinct.get((height, round_, PRECOMMIT), 0) == q,
        "skip": tally.distinct_any.get((height, round_), 0) + (1 if propose_signer_new else 0) >= f + 1,
        "precommit_value": False,
        "commit": False,
        "prevote_validround": False,
    }
    if propose_value is not None and propose_valid:
        out["precommit_value"] = pv(propose_value) >= q
        out["commit"] = pc(propose_value) >= q
    if propose_value is not None and propose_valid_round > INVALID_ROUND:
        out["prevote_validround"] = count.get((height, propose_valid_round, PREVOTE, propose_value), 0) >= q
    return out


def decide_votes(votes, round_: int, f: int, propose_value: Optional[bytes] = None, propose_valid: bool = False,
                 propose_valid_round: int = INVALID_ROUND) -> Dict[str, bool]:
    """The same predicates as :func:`decide`, for the current height of an
    incremental :class:`hyperdrive_amd.votes.VoteLog` (include/hd_votes.h):
    every value is one O(1) lookup where process.go runs its O(n) loops.  A
    valid propose's signer is already in the log's trace (trace_propose)."""
    q = 2 * f + 1
    out = {
        "timeout_prevote": votes.len(PREVOTE, round_) >= q,                 # process.go:534
        "precommit_nil": votes.count(PREVOTE, round_, NIL_VALUE) >= q,     # 626-632
        "timeout_precommit_reached": votes.len(PRECOMMIT, round_) >= q,    # 658 (crossed at some insert)
        "timeout_precommit_exact": votes.len(PRECOMMIT, round_) == q,      # 310 + 658 (StartRound's ==)
        "skip": votes.trace_len(round_) >= f + 1,                          # 751
        "precommit_value": False,
        "commit": False,
        "prevote_validround": False,
    }
    if propose_value is not None and propose_valid:
        out["precommit_value"] = votes.count(PREVOTE, round_, propose_value) >= q     # 574-582
        out["commit"] = votes.count(PRECOMMIT, round_, propose_value) >= q            # 696-702
    if propose_value is not None and propose_valid_round > INVALID_ROUND:
        out["prevote_validround"] = votes.count(PREVOTE, propose_valid_round, propose_value) >= q  # 486-494
    return out
