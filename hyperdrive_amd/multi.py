"""One batch verified and tallied on several GPUs of one process
(include/hd_verify.h hd_multi_*): the C-ABI form of the multi-GPU path, for a
caller that owns several devices (a cgo Replica).  bench.py's N > 1 runs use
one process per GPU over torch.distributed instead (hyperdrive_amd/shard.py);
both shard by message index, all-gather the valid bitmaps over RCCL and
partition the tally by round.

    m = MultiVerifier([0, 1, 2, 3])
    m.set_signatories(sigs)
    res, tally = m.process_batch(batch)       # == Verifier.process_batch(batch)
"""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence, Tuple

import numpy as np

from . import _lib
from ._lib import HDError
from .verify import Batch, TallyResult, VerifyResult, Verifier, _as_rows, _ptr


class MultiVerifier:
    def __init__(self, devices: Sequence[int], compressed=True):
        self._lib = _lib.load()
        devs = np.ascontiguousarray(np.asarray(list(devices), np.int32))
        h = ctypes.c_void_p()
        rc = self._lib.hd_multi_create(len(devs), _ptr(devs), ctypes.byref(h))
        if rc != 0:
            raise HDError(rc, "hd_multi_create")
        self._m = h
        self._close_rank = 1
        _lib.track(self)
        self.devices = [int(d) for d in devs]
        self._check(self._lib.hd_multi_set_pubkey_format(self._m, int(compressed)), "hd_multi_set_pubkey_format")

    def _check(self, rc: int, where: str):
        if rc != 0:
            ctx = self._lib.hd_multi_ctx(self._m, 0) if getattr(self, "_m", None) else None
            detail = self._lib.hd_ctx_last_error(ctx).decode() if ctx else ""
            raise HDError(rc, where, detail)

    def close(self):
        if getattr(self, "_m", None):
            self._lib.hd_multi_destroy(self._m)
            self._m = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def uses_rccl(self) -> bool:
        n, r = ctypes.c_int(), ctypes.c_int()
        self._check(self._lib.hd_multi_size(self._m, ctypes.byref(n), ctypes.byref(r)), "hd_multi_size")
        return bool(r.value)

    def set_signatories(self, signatories) -> None:
        arr = _as_rows(signatories, 32)
        self._check(self._lib.hd_multi_set_signatories(self._m, _ptr(arr), len(arr)), "hd_multi_set_signatories")

    def fastpath_stats(self, k: int = 0) -> Tuple[int, int]:
        known, fb = ctypes.c_uint32(), ctypes.c_uint32()
        ctx = self._lib.hd_multi_ctx(self._m, k)
        self._check(self._lib.hd_ctx_fastpath_stats(ctx, ctypes.byref(known), ctypes.byref(fb)),
                    "hd_ctx_fastpath_stats")
        return known.value, fb.value

    def process_batch(self, batch: Batch, tally: bool = True) -> Tuple[VerifyResult, Optional[TallyResult]]:
        n = len(batch)
        verdict = np.zeros(n, np.uint8)
        rec = np.zeros((n, 32), np.uint8)
        bitmap = np.zeros((n + 31) // 32, np.uint32)
        t, a = Verifier._tally_struct(n)
        cb = batch.c_struct()
        self._check(self._lib.hd_multi_verify_batch(self._m, ctypes.byref(cb), _ptr(verdict), _ptr(rec),
                                                    _ptr(bitmap), ctypes.byref(t) if tally else None),
                    "hd_multi_verify_batch")
        res = VerifyResult(verdict, rec, bitmap)
        return res, (Verifier._tally_result(batch, t, a) if tally else None)


__all__ = ["MultiVerifier"]
