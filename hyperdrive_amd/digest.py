"""Batch digest lanes (include/hd_digest.h).

    d = digest_device(v, KECCAK256, dbatch)            # [n, 32] uint8 on the GPU
    h = hash_bytes_device(v, SHA3_256, data, offsets)  # n byte strings
    verify_digest_device(v, dbatch, d, d_verdict, ...) # recover over given digests

SHA256 is the reference's message digest (id.NewHash); KECCAK256 is
Ethereum's legacy Keccak-256 (pad 0x01); SHA3_256 is FIPS 202 (pad 0x06).
"""
from __future__ import annotations

import ctypes
from typing import Optional

from . import _lib
from .device import DeviceBatch, _torch, work_stream
from .verify import Verifier

SHA256, KECCAK256, SHA3_256 = 0, 1, 2


def _check(v: Verifier, rc: int, where: str):
    if rc != 0:
        lib = _lib.load()
        raise _lib.HDError(rc, where, lib.hd_ctx_last_error(v.handle).decode())


def digest_device(v: Verifier, algo: int, batch: DeviceBatch, out=None, stream=None):
    """Preimage digests of every message of a device batch (zeros for types
    outside Propose/Prevote/Precommit).  Enqueued on `stream` (default: the
    library's work stream); torch's current stream is made to wait for it."""
    torch = _torch()
    dev = batch.height.device
    if out is None:
        out = torch.empty((max(batch.n, 1), 32), dtype=torch.uint8, device=dev)
    ws = stream or work_stream(dev)
    ws.wait_stream(torch.cuda.current_stream(ws.device))
    cs = batch.c_struct()
    _check(v, _lib.load().hd_digest_batch_device(v.handle, algo, ctypes.byref(cs), out.data_ptr(), ws.cuda_stream),
           "hd_digest_batch_device")
    torch.cuda.current_stream(ws.device).wait_stream(ws)   # later torch work sees the digests
    return out[: batch.n]


def hash_bytes_device(v: Verifier, algo: int, data, offsets, out=None, stream=None):
    """algo(data[offsets[i]:offsets[i+1]]) for every i; data a uint8 device
    tensor, offsets an int64 device tensor of n+1 non-decreasing offsets."""
    torch = _torch()
    n = offsets.numel() - 1
    dev = offsets.device
    if out is None:
        out = torch.empty((max(n, 1), 32), dtype=torch.uint8, device=dev)
    ws = stream or work_stream(dev)
    ws.wait_stream(torch.cuda.current_stream(ws.device))
    _check(v, _lib.load().hd_hash_bytes_device(v.handle, algo, data.data_ptr() if data.numel() else None,
                                               offsets.data_ptr(), n, out.data_ptr(), ws.cuda_stream),
           "hd_hash_bytes_device")
    torch.cuda.current_stream(ws.device).wait_stream(ws)
    return out[:n]


def verify_digest_device(v: Verifier, batch: DeviceBatch, digest, d_verdict: int, d_recovered: Optional[int] = None,
                         d_signer: Optional[int] = None, d_bitmap: Optional[int] = None, stream=None) -> None:
    """hd_verify_batch_digest_device: recovery over caller-supplied digests."""
    torch = _torch()
    ws = stream or work_stream(batch.height.device)
    ws.wait_stream(torch.cuda.current_stream(ws.device))
    cs = batch.c_struct()
    _check(v, _lib.load().hd_verify_batch_digest_device(v.handle, ctypes.byref(cs), digest.data_ptr(), d_verdict,
                                                        d_recovered, d_signer, d_bitmap, ws.cuda_stream),
           "hd_verify_batch_digest_device")
    torch.cuda.current_stream(ws.device).wait_stream(ws)
