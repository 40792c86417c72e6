"""Bulk MessageQueue on the GPU (include/hd_mq.h; mq/mq.go).

    q = MessageQueue(verifier, max_capacity=1000)      # mq.New
    q.insert_device(dbatch)                            # InsertPrevote/... for a whole batch (queue = From)
    q.insert_verified_device(dbatch, verdict, h)       # Replica.Run ingress: authenticated, filterHeight
    msgs, senders = q.consume(height, allowed)         # Consume(h, ..., procsAllowed)
    q.drop_below(height)                               # DropMessagesBelowHeight

Queues are keyed by the message's From (mq.go:107-113); ``allowed`` is
procsAllowed, applied at consume time (mq.go:49-51): a list / array of
32-byte signatories, or None for the verifier's current admitted set.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Tuple

import numpy as np

from . import _lib
from ._lib import HdBatchOut
from .device import DeviceBatch, _torch, work_stream
from .verify import Batch, Verifier


def _sig_array(allowed) -> np.ndarray:
    if isinstance(allowed, np.ndarray):
        a = np.ascontiguousarray(allowed, dtype=np.uint8).reshape(-1, 32)
    else:
        a = np.frombuffer(b"".join(bytes(x) for x in allowed), dtype=np.uint8).reshape(-1, 32)
    return np.ascontiguousarray(a)


class MessageQueue:
    def __init__(self, v: Verifier, max_capacity: int = 1000):
        self._v = v
        self._lib = _lib.load()
        h = ctypes.c_void_p()
        rc = self._lib.hd_mq_create(v.handle, max_capacity, ctypes.byref(h))
        if rc != 0:
            raise _lib.HDError(rc, "hd_mq_create")
        self._q = h
        self.max_capacity = max_capacity
        self.last_removed = 0        # Consume's n (delivered + dropped by procsAllowed) of the last consume
        self.inserts = 0             # insert calls so far (lets a caller know the pool is unchanged)
        _lib.track(self)

    def close(self):
        if getattr(self, "_q", None):
            self._lib.hd_mq_destroy(self._q)
            self._q = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc: int, where: str):
        if rc != 0:
            raise _lib.HDError(rc, where, self._lib.hd_ctx_last_error(self._v.handle).decode())

    def insert_device(self, batch: DeviceBatch, insert=None, stream=None) -> None:
        """Insert every message i with insert[i] != 0 (a uint8/bool device
        tensor; None = all), in batch order, into the queue of its From."""
        torch = _torch()
        ws = stream or work_stream(batch.height.device)
        ws.wait_stream(torch.cuda.current_stream(ws.device))
        cs = batch.c_struct()
        ptr = None
        if insert is not None:
            if insert.dtype == torch.bool:
                insert = insert.to(torch.uint8)
            ptr = insert.data_ptr()
        self.inserts += 1
        self._check(self._lib.hd_mq_insert_device(self._q, ctypes.byref(cs), ptr, ws.cuda_stream),
                    "hd_mq_insert_device")

    def insert_verified_device(self, batch: DeviceBatch, verdict, min_height: int, stream=None) -> None:
        """Replica ingress: insert the authenticated messages (verdict VALID or
        NOT_ADMITTED) with height >= min_height (filterHeight); membership is
        checked at consume time."""
        torch = _torch()
        ws = stream or work_stream(batch.height.device)
        ws.wait_stream(torch.cuda.current_stream(ws.device))
        cs = batch.c_struct()
        self.inserts += 1
        self._check(self._lib.hd_mq_insert_verified_device(self._q, ctypes.byref(cs), verdict.data_ptr(),
                                                           int(min_height), ws.cuda_stream),
                    "hd_mq_insert_verified_device")

    def __len__(self) -> int:
        n = ctypes.c_uint64()
        self._check(self._lib.hd_mq_size(self._q, ctypes.byref(n)), "hd_mq_size")
        return int(n.value)

    @property
    def senders(self) -> int:
        """Sender queues created so far (distinct Froms ever inserted)."""
        n = ctypes.c_uint32()
        self._check(self._lib.hd_mq_senders(self._q, ctypes.byref(n)), "hd_mq_senders")
        return int(n.value)

    def _out_arrays(self, n: int):
        """Host arrays for up to n delivered messages, reused across consumes
        (grown on demand): a flush delivers a few messages per sender, the
        queue may hold a million."""
        if getattr(self, "_cap", 0) < n:
            n = max(n, 2 * getattr(self, "_cap", 0), 1024)
            self._a = dict(type=np.empty(n, np.uint8), height=np.empty(n, np.int64), round=np.empty(n, np.int64),
                           valid_round=np.empty(n, np.int64), value=np.empty((n, 32), np.uint8),
                           frm=np.empty((n, 32), np.uint8), sig=np.empty((n, 65), np.uint8))
            self._snd = np.empty(n, np.int32)
            p = lambda x: x.ctypes.data
            a = self._a
            self._out = HdBatchOut(p(a["type"]), p(a["height"]), p(a["round"]), p(a["valid_round"]), p(a["value"]),
                                   p(a["frm"]), p(a["sig"]), None)
            self._out_ref = ctypes.byref(self._out)
            self._snd_p = p(self._snd)
            self._cap = n
        return self._a, self._snd, self._out

    def consume(self, height: int, allowed=None) -> Tuple[Batch, np.ndarray]:
        """Remove every message with height <= `height`; return those of
        senders in `allowed` (procsAllowed; None = the verifier's admitted set
        now), sender queues in creation order, each by (height, round,
        arrival), with their sender-queue ids.  ``last_removed`` is set to the
        number removed, delivered or not."""
        p = lambda x: x.ctypes.data
        got, removed = ctypes.c_uint32(), ctypes.c_uint32()
        if allowed is None:
            al, na = None, 0
        else:
            arr = _sig_array(allowed)
            al, na = (p(arr) if len(arr) else p(np.zeros((1, 32), np.uint8))), len(arr)
        a, snd, out = self._out_arrays(1024)
        while True:
            rc = self._lib.hd_mq_consume(self._q, int(height), al, na, ctypes.byref(out), p(snd), self._cap,
                                         ctypes.byref(got), ctypes.byref(removed))
            if rc != _lib.HD_ECAP:
                break
            a, snd, out = self._out_arrays(int(got.value))     # nothing was removed: retry with room
        self._check(rc, "hd_mq_consume")
        k = int(got.value)
        self.last_removed = int(removed.value)
        b = Batch(a["type"][:k].copy(), a["height"][:k].copy(), a["round"][:k].copy(), a["valid_round"][:k].copy(),
                  a["value"][:k].copy(), a["frm"][:k].copy(), a["sig"][:k].copy())
        return b, snd[:k].copy()

    def consume_votes(self, height: int, votes) -> Tuple[Batch, np.ndarray, np.ndarray, np.ndarray, np.ndarray]:
        """consume(height) with procsAllowed = the verifier's admitted set,
        and the delivered messages inserted into the vote logs `votes`
        (votes.VoteLog) in the same foreign call (include/hd_mq.h
        hd_mq_consume_votes).  Returns (batch, senders, status, double_of,
        events), each per delivered message."""
        # (a flush is ~25 us of foreign call: the counters, their byrefs and
        # the buffers' addresses are made once, not per call)
        if getattr(self, "_cnt", None) is None:
            self._cnt = (ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32())
            self._cnt_ref = tuple(ctypes.byref(c) for c in self._cnt)
        got, removed, ins = self._cnt
        r_got, r_removed, r_ins = self._cnt_ref
        a, snd, out = self._out_arrays(1024)
        while True:
            st, dbl, ev = self._vote_arrays()
            vp = self._vote_ptrs
            rc = self._lib.hd_mq_consume_votes(self._q, votes._v, int(height), None, 0, self._out_ref, self._snd_p,
                                               self._cap, r_got, r_removed, vp[0], vp[1], vp[2], r_ins)
            if rc != _lib.HD_ECAP:
                break
            a, snd, out = self._out_arrays(int(got.value))
        self._check(rc, "hd_mq_consume_votes")
        k = int(got.value)
        self.last_removed = int(removed.value)
        b = Batch._wrap(a["type"][:k].copy(), a["height"][:k].copy(), a["round"][:k].copy(),
                        a["valid_round"][:k].copy(), a["value"][:k].copy(), a["frm"][:k].copy(), a["sig"][:k].copy())
        return b, snd[:k].copy(), st[:k].copy(), dbl[:k].copy(), ev[:k].copy()

    def _vote_arrays(self):
        if getattr(self, "_vcap", 0) < self._cap:
            self._vst = np.empty(self._cap, np.uint8)
            self._vdbl = np.empty(self._cap, np.uint32)
            self._vev = np.empty(self._cap, np.uint8)
            self._vote_ptrs = (self._vst.ctypes.data, self._vdbl.ctypes.data, self._vev.ctypes.data)
            self._vcap = self._cap
        return self._vst, self._vdbl, self._vev

    def drop_below(self, height: int) -> None:
        self._check(self._lib.hd_mq_drop_below(self._q, int(height)), "hd_mq_drop_below")
