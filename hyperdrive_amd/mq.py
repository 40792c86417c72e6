"""Bulk MessageQueue on the GPU (include/hd_mq.h; mq/mq.go).

    q = MessageQueue(verifier, max_capacity=1000)      # mq.New
    q.insert_device(dbatch, d_sender)                  # InsertPrevote/... for a whole batch
    msgs, senders = q.consume(height)                  # Consume(h): host Batch + sender ids
    q.drop_below(height)                               # DropMessagesBelowHeight
"""
from __future__ import annotations

import ctypes
from typing import Tuple

import numpy as np

from . import _lib
from ._lib import HdBatchOut
from .device import DeviceBatch, _torch, work_stream
from .verify import Batch, Verifier


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

    def insert_device(self, batch: DeviceBatch, sender, stream=None) -> None:
        """Insert every message i with sender[i] >= 0 (an int32 device tensor), in
        batch order."""
        torch = _torch()
        ws = stream or work_stream(batch.height.device)
        ws.wait_stream(torch.cuda.current_stream(ws.device))
        cs = batch.c_struct()
        self._check(self._lib.hd_mq_insert_device(self._q, ctypes.byref(cs), sender.data_ptr(), ws.cuda_stream),
                    "hd_mq_insert_device")

    def insert_verified_device(self, batch: DeviceBatch, verdict, signer, min_height: int, stream=None) -> None:
        """Replica ingress: insert the VALID messages with height >= min_height
        (filterHeight), sender = signer[i] (device tensors from verify)."""
        torch = _torch()
        ws = stream or work_stream(batch.height.device)
        ws.wait_stream(torch.cuda.current_stream(ws.device))
        cs = batch.c_struct()
        self._check(self._lib.hd_mq_insert_verified_device(self._q, ctypes.byref(cs), verdict.data_ptr(),
                                                           signer.data_ptr(), int(min_height), ws.cuda_stream),
                    "hd_mq_insert_verified_device")

    def __len__(self) -> int:
        n = ctypes.c_uint64()
        self._check(self._lib.hd_mq_size(self._q, ctypes.byref(n)), "hd_mq_size")
        return int(n.value)

    def consume(self, height: int) -> Tuple[Batch, np.ndarray]:
        """Remove and return every message with height <= `height`, senders
        ascending, each sender's messages by (height, round, arrival)."""
        cap = len(self)
        n = max(cap, 1)
        a = dict(type=np.zeros(n, np.uint8), height=np.zeros(n, np.int64), round=np.zeros(n, np.int64),
                 valid_round=np.zeros(n, np.int64), value=np.zeros((n, 32), np.uint8),
                 frm=np.zeros((n, 32), np.uint8), sig=np.zeros((n, 65), np.uint8))
        snd = np.zeros(n, np.int32)
        p = lambda x: x.ctypes.data
        out = HdBatchOut(p(a["type"]), p(a["height"]), p(a["round"]), p(a["valid_round"]), p(a["value"]),
                         p(a["frm"]), p(a["sig"]), None)
        got = ctypes.c_uint32()
        self._check(self._lib.hd_mq_consume(self._q, int(height), ctypes.byref(out), p(snd), cap, ctypes.byref(got)),
                    "hd_mq_consume")
        k = int(got.value)
        b = Batch(a["type"][:k], a["height"][:k], a["round"][:k], a["valid_round"][:k], a["value"][:k], a["frm"][:k],
                  a["sig"][:k])
        return b, snd[:k].copy()

    def drop_below(self, height: int) -> None:
        self._check(self._lib.hd_mq_drop_below(self._q, int(height)), "hd_mq_drop_below")
