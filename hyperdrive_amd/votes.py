"""Incremental vote logs and count table of one height (include/hd_votes.h).

The state a Process keeps for its current height (process/state.go:44-57),
with per-value vote counts maintained on insert so that the rule checks of
process.go (L28/L36/L44/L47/L49/L55) are O(1) lookups instead of O(n) loops:

    v = VoteLog(height)
    v.insert(PREVOTE, h, r, value, frm)      # insertPrevote -> (status, logged value)
    v.insert_batch(batch, verdict)           # a verified batch in arrival order
    v.trace_propose(r, frm)                  # valid propose signer -> TraceLogs
    v.count(PREVOTE, r, value); v.len(PRECOMMIT, r); v.trace_len(r)
    v.reset(h + 1)                           # new height (process.go:718-724)

With ``set_f(f)``, each insert also reports the thresholds it made a log reach
exactly (``last_events``; EV_PRECOMMIT_2F1 is L47's equality crossing,
process.go:658).
"""
from __future__ import annotations

import ctypes
from typing import Optional, Tuple

import numpy as np

from . import _lib
from .verify import PRECOMMIT, PREVOTE, Batch, _ptr

INSERTED, WRONG_HEIGHT, DUPLICATE, DOUBLE, NOT_VOTE, SKIPPED = range(6)
EV_PREVOTE_2F1, EV_PRECOMMIT_2F1, EV_TRACE_F1 = 1, 2, 4     # include/hd_votes.h HD_VOTE_EV_*
STATUS_NAMES = ["INSERTED", "WRONG_HEIGHT", "DUPLICATE", "DOUBLE", "NOT_VOTE", "SKIPPED"]
NO_INDEX = 0xFFFFFFFF


def _b32(x) -> bytes:
    b = bytes(x)
    if len(b) != 32:
        raise ValueError("value / signatory must be 32 bytes")
    return b


class VoteLog:
    def __init__(self, height: int = 0):
        self._lib = _lib.load()
        h = ctypes.c_void_p()
        self._check(self._lib.hd_votes_create(int(height), ctypes.byref(h)), "hd_votes_create")
        self._v = h
        self.last_events = 0      # HD_VOTE_EV_* of the last insert / trace_propose (array after insert_batch)
        _lib.track(self)

    def _check(self, rc: int, where: str):
        if rc != 0:
            raise _lib.HDError(rc, where)

    def close(self):
        if getattr(self, "_v", None):
            self._lib.hd_votes_destroy(self._v)
            self._v = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def height(self) -> int:
        h = ctypes.c_int64()
        self._check(self._lib.hd_votes_height(self._v, ctypes.byref(h)), "hd_votes_height")
        return h.value

    def set_f(self, f: int) -> None:
        """f for the quorum-crossing events (len(signatories) // 3)."""
        self._check(self._lib.hd_votes_set_f(self._v, int(f)), "hd_votes_set_f")

    def reset(self, height: int) -> None:
        self._check(self._lib.hd_votes_reset(self._v, int(height)), "hd_votes_reset")

    def insert(self, mtype: int, height: int, round_: int, value, frm) -> Tuple[int, Optional[bytes]]:
        """(status, logged value if status == DOUBLE else None)."""
        st, ev = ctypes.c_uint8(), ctypes.c_uint8()
        prev = ctypes.create_string_buffer(32)
        self._check(self._lib.hd_votes_insert(self._v, mtype, int(height), int(round_), _b32(value), _b32(frm),
                                              ctypes.byref(st), prev, ctypes.byref(ev)), "hd_votes_insert")
        self.last_events = ev.value
        return st.value, (prev.raw if st.value == DOUBLE else None)

    def insert_batch(self, batch: Batch, verdict: Optional[np.ndarray] = None) -> Tuple[np.ndarray, np.ndarray]:
        """Insert the batch's VALID votes in batch order; returns (status[n],
        double_of[n]) -- double_of is the batch index of the logged vote a
        DOUBLE conflicts with, or NO_INDEX if that vote came from an earlier call."""
        n = len(batch)
        status = np.zeros(n, np.uint8)
        double_of = np.zeros(n, np.uint32)
        events = np.zeros(n, np.uint8)
        if verdict is not None:
            verdict = np.ascontiguousarray(verdict, np.uint8)
            if len(verdict) != n:
                raise ValueError("verdict length mismatch")
        cs = batch.c_struct()
        ins = ctypes.c_uint32()
        self._check(self._lib.hd_votes_insert_batch(self._v, ctypes.byref(cs), _ptr(verdict), _ptr(status),
                                                    _ptr(double_of), _ptr(events), ctypes.byref(ins)),
                    "hd_votes_insert_batch")
        self.last_events = events
        return status, double_of

    def trace_propose(self, round_: int, frm) -> None:
        ev = ctypes.c_uint8()
        self._check(self._lib.hd_votes_trace_propose(self._v, int(round_), _b32(frm), ctypes.byref(ev)),
                    "hd_votes_trace_propose")
        self.last_events = ev.value

    def count(self, mtype: int, round_: int, value) -> int:
        n = ctypes.c_uint32()
        self._check(self._lib.hd_votes_count(self._v, mtype, int(round_), _b32(value), ctypes.byref(n)),
                    "hd_votes_count")
        return n.value

    def len(self, mtype: int, round_: int) -> int:
        n = ctypes.c_uint32()
        self._check(self._lib.hd_votes_len(self._v, mtype, int(round_), ctypes.byref(n)), "hd_votes_len")
        return n.value

    def trace_len(self, round_: int) -> int:
        n = ctypes.c_uint32()
        self._check(self._lib.hd_votes_trace_len(self._v, int(round_), ctypes.byref(n)), "hd_votes_trace_len")
        return n.value

    def get(self, mtype: int, round_: int, frm) -> Optional[bytes]:
        buf = ctypes.create_string_buffer(32)
        found = ctypes.c_int()
        self._check(self._lib.hd_votes_get(self._v, mtype, int(round_), _b32(frm), buf, ctypes.byref(found)),
                    "hd_votes_get")
        return buf.raw if found.value else None


__all__ = ["VoteLog", "PREVOTE", "PRECOMMIT", "INSERTED", "WRONG_HEIGHT", "DUPLICATE", "DOUBLE", "NOT_VOTE",
           "SKIPPED", "NO_INDEX", "STATUS_NAMES", "EV_PREVOTE_2F1", "EV_PRECOMMIT_2F1", "EV_TRACE_F1"]
