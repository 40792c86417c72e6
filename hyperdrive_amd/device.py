"""Device-resident batches (HBM) for the *_device entry points.

PyTorch is used only as plumbing here: it owns the HBM allocations and the
stream the kernels are enqueued on.  All compute is the HIP library.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Optional

import numpy as np

from . import _lib
from ._lib import HdBatch, HdBatchOut
from .verify import Batch, Verifier


def _torch():
    import torch
    return torch


_STREAMS = {}


def work_stream(device=None, priority: int = 0):
    """A dedicated (non-default) torch stream per device for library launches.

    The C ABI reads a NULL stream as "the context's own stream", and torch's
    default stream has handle 0, so device work is always enqueued on an
    explicit stream whose handle is non-zero.  `priority` (torch convention:
    lower is higher, -1 = high) applies when the stream is first created: a
    high-priority verify stream keeps its workgroups ahead of side work (the
    tally of an earlier batch) queued on normal streams."""
    return verify_streams(device, 1, priority)[0]


def verify_streams(device=None, k: int = 2, priority: int = 0):
    """work_stream(device) and the streams that verify beside it, k in all,
    created together when the work stream is first made.  The runtime maps
    streams onto the device's few hardware queues (GPU_MAX_HW_QUEUES, 4) round
    robin in creation order, so streams created one after another get
    different queues; a verify stream created later (after a tally stream, or
    by another component) may share the work stream's queue and serialise
    behind its kernels (the C5 ingress inside bench.py: push 2.84 ms against
    2.30 ms standalone).  Every component that verifies beside the work
    stream (bench.Pipeline, Ingress.push_wires) takes its streams from here."""
    torch = _torch()
    dev = torch.device("cuda", torch.cuda.current_device() if device is None else torch.device(device).index or 0)
    have = _STREAMS.setdefault(dev, [])
    if not have:
        have.extend(torch.cuda.Stream(device=dev, priority=priority) for _ in range(max(k, 3)))
    while len(have) < k:
        have.append(torch.cuda.Stream(device=dev, priority=have[0].priority))
    return have[:k]


@dataclass
class DeviceBatch:
    n: int
    type: "object"
    height: "object"
    round: "object"
    valid_round: "object"
    value: "object"
    frm: "object"
    sig: "object"
    adv_class: "object" = None

    @classmethod
    def empty(cls, n: int, device: str = "cuda") -> "DeviceBatch":
        torch = _torch()
        u8, i64 = torch.uint8, torch.int64
        return cls(n, torch.empty(n, dtype=u8, device=device), torch.empty(n, dtype=i64, device=device),
                   torch.empty(n, dtype=i64, device=device), torch.empty(n, dtype=i64, device=device),
                   torch.empty((n, 32), dtype=u8, device=device), torch.empty((n, 32), dtype=u8, device=device),
                   torch.empty((n, 65), dtype=u8, device=device), torch.empty(n, dtype=torch.int8, device=device))

    @classmethod
    def from_host(cls, b: Batch, device: str = "cuda") -> "DeviceBatch":
        torch = _torch()
        vr = b.valid_round if b.valid_round is not None else np.full(len(b), -1, np.int64)
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)
        return cls(len(b), t(b.type), t(b.height), t(b.round), t(vr), t(b.value), t(b.frm), t(b.sig))

    def rows(self, lo: int, n: int) -> "DeviceBatch":
        """Rows lo .. lo + n - 1 as views (no copy)."""
        f = lambda t: t[lo: lo + n] if t is not None else None
        return DeviceBatch(n, f(self.type), f(self.height), f(self.round), f(self.valid_round), f(self.value),
                           f(self.frm), f(self.sig), f(self.adv_class))

    def c_struct(self) -> HdBatch:
        return HdBatch(self.n, self.type.data_ptr(), self.height.data_ptr(), self.round.data_ptr(),
                       self.valid_round.data_ptr(), self.value.data_ptr(), self.frm.data_ptr(), self.sig.data_ptr())

    def c_out(self) -> HdBatchOut:
        return HdBatchOut(self.type.data_ptr(), self.height.data_ptr(), self.round.data_ptr(),
                          self.valid_round.data_ptr(), self.value.data_ptr(), self.frm.data_ptr(),
                          self.sig.data_ptr(), self.adv_class.data_ptr() if self.adv_class is not None else None)

    def to_host(self) -> Batch:
        c = lambda t: t.cpu().numpy()
        return Batch(c(self.type), c(self.height), c(self.round), c(self.valid_round), c(self.value), c(self.frm),
                     c(self.sig))


def generate(v: Verifier, kind: int, n: int, S: int, adv_pct: int = 0, start: int = 0,
             keys=None, stream: Optional[int] = None, device: str = "cuda"):
    """Seeded synthetic workload generated on the GPU (hd_gen_batch_device).
    Returns (DeviceBatch, signatories[S,32] numpy, foreign[16,32] numpy)."""
    torch = _torch()
    sigs, foreign = keys if keys is not None else v.gen_keys(S)
    d_sigs = torch.from_numpy(np.ascontiguousarray(sigs)).to(device)
    d_for = torch.from_numpy(np.ascontiguousarray(foreign)).to(device)
    db = DeviceBatch.empty(n, device)
    out = db.c_out()
    lib = _lib.load()
    ws = work_stream(device)
    ws.wait_stream(torch.cuda.current_stream(ws.device))
    rc = lib.hd_gen_batch_device(v.handle, kind, start, n, S, adv_pct, d_sigs.data_ptr(), d_for.data_ptr(),
                                 ctypes.byref(out), stream if stream else ws.cuda_stream)
    if rc != 0:
        raise _lib.HDError(rc, "hd_gen_batch_device", lib.hd_ctx_last_error(v.handle).decode())
    ws.synchronize()
    return db, sigs, foreign
