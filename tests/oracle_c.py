"""ctypes face of the C oracle (oracle/hd_oracle.c) -- test infrastructure."""
from __future__ import annotations

import ctypes

import numpy as np


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


class COracle:
    def __init__(self, path: str):
        self.lib = ctypes.CDLL(path)
        self.lib.oracle_verify_batch.restype = ctypes.c_int
        self.lib.oracle_verify_batch.argtypes = [ctypes.c_uint32] + [ctypes.c_void_p] * 8 + [
            ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        self.lib.oracle_sha256.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_void_p]
        self.lib.oracle_recover.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_void_p]
        self.lib.oracle_recover.restype = ctypes.c_int
        self.lib.oracle_digest.argtypes = [ctypes.c_uint8, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                           ctypes.c_char_p, ctypes.c_void_p]
        self.lib.oracle_tally.restype = ctypes.c_int
        self.lib.oracle_tally.argtypes = [ctypes.c_uint32] + [ctypes.c_void_p] * 6 + [ctypes.c_uint32, ctypes.c_void_p,
                                                                                      ctypes.c_void_p, ctypes.c_void_p,
                                                                                      ctypes.c_void_p, ctypes.c_void_p,
                                                                                      ctypes.c_void_p]

    def sha256(self, b: bytes) -> bytes:
        out = ctypes.create_string_buffer(32)
        self.lib.oracle_sha256(b, len(b), out)
        return out.raw

    def digest(self, t, h, r, vr, value) -> bytes:
        out = ctypes.create_string_buffer(32)
        self.lib.oracle_digest(t, h, r, vr, value, out)
        return out.raw

    def recover(self, digest: bytes, sig: bytes):
        out = ctypes.create_string_buffer(65)
        v = self.lib.oracle_recover(digest, sig, out)
        return v, (out.raw if v == 0 else None)

    def verify(self, batch, admitted: np.ndarray, compressed: bool = True, threads: int = 1):
        """batch: hyperdrive_amd.verify.Batch (numpy SoA).  Returns (verdict, recovered)."""
        n = len(batch)
        verdict = np.zeros(n, np.uint8)
        rec = np.zeros((n, 32), np.uint8)
        adm = np.ascontiguousarray(admitted, dtype=np.uint8).reshape(-1, 32)
        rc = self.lib.oracle_verify_batch(n, _p(batch.type), _p(batch.height), _p(batch.round),
                                          _p(batch.valid_round), _p(batch.value), _p(batch.frm), _p(batch.sig),
                                          _p(adm), len(adm), int(compressed), _p(verdict), _p(rec), threads)
        assert rc == 0
        return verdict, rec

    def tally(self, batch, verdict, f: int = 0, pv_by_hr=None, propose_value=None):
        """First-wins tally + quorum decisions (oracle_tally).  Returns
        {"counts": [k, 5] int64 (h, r, type, rep, n), "hr": [m, 6] int64 (h, r,
        prevotes, precommits, any, rep), "decide": [m] uint8 bits}.
        propose_value(h, r) -> 32 bytes or None gives the propose value of each
        round (else pv_by_hr, else no propose)."""
        n = len(batch)
        verdict = np.ascontiguousarray(verdict, np.uint8)
        counts = np.zeros((max(n, 1), 5), np.int64)
        hr = np.zeros((max(n, 1), 6), np.int64)
        nc, nh = ctypes.c_uint32(), ctypes.c_uint32()
        rc = self.lib.oracle_tally(n, _p(batch.type), _p(batch.height), _p(batch.round), _p(batch.value),
                                   _p(batch.frm), _p(verdict), 0, None, _p(counts), ctypes.byref(nc), _p(hr),
                                   ctypes.byref(nh), None)
        assert rc == 0
        hr = hr[: nh.value]
        if propose_value is not None:
            pv_by_hr = np.array([np.frombuffer(propose_value(int(h), int(r)), np.uint8) for h, r in hr[:, :2]],
                                np.uint8).reshape(-1, 32)
        decide = np.zeros(max(nh.value, 1), np.uint8)
        rc = self.lib.oracle_tally(n, _p(batch.type), _p(batch.height), _p(batch.round), _p(batch.value),
                                   _p(batch.frm), _p(verdict), int(f), _p(pv_by_hr), _p(counts), ctypes.byref(nc),
                                   _p(np.zeros((max(n, 1), 6), np.int64)), ctypes.byref(nh), _p(decide))
        assert rc == 0
        return {"counts": counts[: nc.value].copy(), "hr": hr.copy(), "decide": decide[: nh.value].copy()}


class GlvPort:
    """The CPU baseline "port-glv" (oracle/glv_port.cpp): the repository's own
    GLV recovery built for the host, threaded.  Not the oracle; bench.py's
    cpu_baseline leg and its test only."""

    def __init__(self, path: str):
        self.lib = ctypes.CDLL(path)
        self.lib.glv_verify.restype = ctypes.c_int
        self.lib.glv_verify.argtypes = [ctypes.c_uint32] + [ctypes.c_void_p] * 8 + [ctypes.c_uint32, ctypes.c_int] + \
            [ctypes.c_void_p] * 3 + [ctypes.c_int]

    def verify(self, batch, admitted: np.ndarray, compressed: bool = True, threads: int = 1):
        n = len(batch)
        verdict = np.zeros(n, np.uint8)
        rec = np.zeros((n, 32), np.uint8)
        adm = np.ascontiguousarray(admitted, dtype=np.uint8).reshape(-1, 32)
        rc = self.lib.glv_verify(n, _p(batch.type), _p(batch.height), _p(batch.round), _p(batch.valid_round),
                                 _p(batch.value), _p(batch.frm), _p(batch.sig), _p(adm), len(adm), int(compressed),
                                 _p(verdict), _p(rec), None, threads)
        assert rc == 0
        return verdict, rec


class SecpPort:
    """The CPU baseline "port-secp-class" (oracle/secp_port.cpp): a C++
    restatement of the reference path in libsecp256k1's algorithm class
    (5 x 52-bit field, GLV + wNAF Strauss ladder, precomputed G table,
    divsteps inversions), threaded.  Not the oracle; bench.py's cpu_baseline
    leg and its test only."""

    def __init__(self, path: str):
        self.lib = ctypes.CDLL(path)
        self.lib.secp_verify.restype = ctypes.c_int
        self.lib.secp_verify.argtypes = [ctypes.c_uint32] + [ctypes.c_void_p] * 8 + [ctypes.c_uint32, ctypes.c_int] + \
            [ctypes.c_void_p] * 3 + [ctypes.c_int]

    def verify(self, batch, admitted: np.ndarray, compressed: bool = True, threads: int = 1):
        n = len(batch)
        verdict = np.zeros(n, np.uint8)
        rec = np.zeros((n, 32), np.uint8)
        adm = np.ascontiguousarray(admitted, dtype=np.uint8).reshape(-1, 32)
        rc = self.lib.secp_verify(n, _p(batch.type), _p(batch.height), _p(batch.round), _p(batch.valid_round),
                                  _p(batch.value), _p(batch.frm), _p(batch.sig), _p(adm), len(adm), int(compressed),
                                  _p(verdict), _p(rec), None, threads)
        assert rc == 0
        return verdict, rec
