"""Batch surge codec of Propose / Prevote / Precommit on the GPU
(include/hd_codec.h; process/message.go Marshal / Unmarshal).

    buf = marshal_device(v, PREVOTE, batch, with_sig=True)     # torch uint8 on the GPU
    batch2, status = unmarshal_device(v, PREVOTE, buf, n, with_sig=True)

PyTorch only owns the HBM buffers; the (de)serialisation is the HIP library.
"""
from __future__ import annotations

import ctypes
from typing import Tuple

from . import _lib
from .device import DeviceBatch, _torch, work_stream
from .verify import Verifier

PROPOSE, PREVOTE, PRECOMMIT = 1, 2, 3


def record_size(mtype: int, with_sig: bool) -> int:
    return int(_lib.load().hd_record_size(mtype, 1 if with_sig else 0))


def marshal_device(v: Verifier, mtype: int, batch: DeviceBatch, with_sig: bool = True, stream=None):
    """Encode every message of a device batch as `mtype` records."""
    torch = _torch()
    s = record_size(mtype, with_sig)
    if s == 0:
        raise ValueError(f"bad message type {mtype}")
    buf = torch.empty(max(batch.n * s, 16), dtype=torch.uint8, device=batch.height.device)
    cs = batch.c_struct()
    lib = _lib.load()
    ws = stream or work_stream(batch.height.device)
    ws.wait_stream(torch.cuda.current_stream(ws.device))
    rc = lib.hd_marshal_batch_device(v.handle, mtype, 1 if with_sig else 0, ctypes.byref(cs), buf.data_ptr(),
                                     buf.numel(), ws.cuda_stream)
    if rc != 0:
        raise _lib.HDError(rc, "hd_marshal_batch_device", lib.hd_ctx_last_error(v.handle).decode())
    ws.synchronize()
    return buf[: batch.n * s]


def unmarshal_device(v: Verifier, mtype: int, buf, n: int, with_sig: bool = True,
                     stream=None, sync: bool = True, out: DeviceBatch = None,
                     wait: bool = True) -> Tuple[DeviceBatch, "object"]:
    """Decode n `mtype` records from a device byte buffer into a DeviceBatch;
    status[i] = 1 marks a record the buffer ended before.  sync=False leaves
    the decode queued on `stream` (the caller orders what reads the batch
    after it on that stream).  out: decode into this batch (n rows, e.g. a
    view into a larger one; its sig rows must start 16-byte aligned).
    wait=False: `stream` does not first wait for the current stream (the
    caller has ordered the buffer's producer before it, e.g. push_wires'
    event: otherwise a second buffer's decode on another stream would queue
    behind the first buffer's verification)."""
    torch = _torch()
    dev = buf.device
    if out is None:
        out = DeviceBatch.empty(n, str(dev))
    status = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
    co = out.c_out()
    lib = _lib.load()
    ws = stream or work_stream(dev)
    if wait:
        ws.wait_stream(torch.cuda.current_stream(ws.device))
    rc = lib.hd_unmarshal_batch_device(v.handle, mtype, 1 if with_sig else 0, buf.data_ptr(), buf.numel(), n,
                                       ctypes.byref(co), status.data_ptr(), ws.cuda_stream)
    if rc != 0:
        raise _lib.HDError(rc, "hd_unmarshal_batch_device", lib.hd_ctx_last_error(v.handle).decode())
    if sync:
        ws.synchronize()
    return out, status[:n]
