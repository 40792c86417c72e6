"""ctypes face of tests/native/hd_host_check.cpp: the device math headers built
for the host (test harness only; never a product fallback)."""
from __future__ import annotations

import ctypes

import numpy as np


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def b32(x: int) -> bytes:
    return x.to_bytes(32, "big")


class HostMath:
    FE_OPS = {"mul": 0, "sqr": 1, "add": 2, "sub": 3, "neg": 4, "inv": 5, "sqrt": 6, "inv_divsteps": 7}
    SC_OPS = {"mul": 0, "sqr": 1, "neg": 2, "inv": 3, "reduce": 4, "inv_divsteps": 5}

    def __init__(self, path: str):
        L = ctypes.CDLL(path)
        self.L = L
        L.hdh_booth.restype = ctypes.c_int
        L.hdh_ecmult.restype = ctypes.c_int
        L.hdh_recover.restype = ctypes.c_int
        L.hdh_gen.argtypes = [ctypes.c_uint32, ctypes.c_uint64] + [ctypes.c_uint32] * 3 + [ctypes.c_void_p] * 10
        L.hdh_verify.argtypes = [ctypes.c_uint32] + [ctypes.c_void_p] * 8 + [ctypes.c_uint32, ctypes.c_int] + \
            [ctypes.c_void_p] * 3

    def fe(self, op: str, a: int, b: int = 0):
        out = ctypes.create_string_buffer(33)
        self.L.hdh_fe_op(self.FE_OPS[op], b32(a), b32(b), out)
        return int.from_bytes(out.raw[:32], "big"), bool(out.raw[32])

    def sc(self, op: str, a: int, b: int = 0) -> int:
        out = ctypes.create_string_buffer(32)
        self.L.hdh_sc_op(self.SC_OPS[op], b32(a), b32(b), out)
        return int.from_bytes(out.raw, "big")

    def gtab(self):
        """256 entries: (k+1) G for k < 128, then lambda (k+1) G."""
        out = ctypes.create_string_buffer(256 * 64)
        self.L.hdh_gtab(out)
        r = out.raw
        return [(int.from_bytes(r[64 * k:64 * k + 32], "big"), int.from_bytes(r[64 * k + 32:64 * k + 64], "big"))
                for k in range(256)]

    def ecmult_glv(self, R, u1: int, u2: int):
        out = ctypes.create_string_buffer(64)
        inf = self.L.hdh_ecmult_glv(b32(R[0]), b32(R[1]), b32(u1), b32(u2), out)
        if inf:
            return None
        return int.from_bytes(out.raw[:32], "big"), int.from_bytes(out.raw[32:], "big")

    def ecmult_glv_fbg8(self, R, u1: int, u2: int):
        """ecmult_glv_fbg over an 8-bit-window fixed-base G table (hd_fixedbase.h)"""
        out = ctypes.create_string_buffer(64)
        inf = self.L.hdh_ecmult_glv_fbg8(b32(R[0]), b32(R[1]), b32(u1), b32(u2), out)
        if inf:
            return None
        return int.from_bytes(out.raw[:32], "big"), int.from_bytes(out.raw[32:], "big")

    def split(self, k: int):
        a = ctypes.create_string_buffer(32)
        b = ctypes.create_string_buffer(32)
        self.L.hdh_split(b32(k), a, b)
        return int.from_bytes(a.raw, "big"), int.from_bytes(b.raw, "big")

    def booth(self, k: int, w: int, j: int) -> int:
        return self.L.hdh_booth(b32(k), w, j)

    def ecmult(self, R, u1: int, u2: int):
        out = ctypes.create_string_buffer(64)
        inf = self.L.hdh_ecmult(b32(R[0]), b32(R[1]), b32(u1), b32(u2), out)
        if inf:
            return None
        return int.from_bytes(out.raw[:32], "big"), int.from_bytes(out.raw[32:], "big")

    def recover(self, digest: bytes, sig: bytes):
        out = ctypes.create_string_buffer(64)
        v = self.L.hdh_recover(digest, sig, out)
        if v != 0:
            return v, None
        return v, (int.from_bytes(out.raw[:32], "big"), int.from_bytes(out.raw[32:], "big"))

    def sign(self, sk: int, digest: bytes) -> bytes:
        out = ctypes.create_string_buffer(65)
        self.L.hdh_sign(b32(sk), digest, out)
        return out.raw

    def signer_sk(self, idx: int) -> int:
        out = ctypes.create_string_buffer(32)
        self.L.hdh_signer_sk(idx, out)
        return int.from_bytes(out.raw, "big")

    def keys(self, S: int, compressed: bool = True):
        sigs = np.zeros((S, 32), np.uint8)
        foreign = np.zeros((16, 32), np.uint8)
        self.L.hdh_keys(S, int(compressed), _p(sigs), _p(foreign))
        return sigs, foreign

    def gen(self, kind: int, start: int, n: int, S: int, adv_pct: int, keys):
        from hyperdrive_amd.verify import Batch
        sigs, foreign = keys
        ty = np.zeros(n, np.uint8)
        h = np.zeros(n, np.int64)
        r = np.zeros(n, np.int64)
        vr = np.zeros(n, np.int64)
        val = np.zeros((n, 32), np.uint8)
        frm = np.zeros((n, 32), np.uint8)
        sg = np.zeros((n, 65), np.uint8)
        cl = np.zeros(n, np.int8)
        self.L.hdh_gen(kind, start, n, S, adv_pct, _p(np.ascontiguousarray(sigs)), _p(np.ascontiguousarray(foreign)),
                       _p(ty), _p(h), _p(r), _p(vr), _p(val), _p(frm), _p(sg), _p(cl))
        return Batch(ty, h, r, vr, val, frm, sg), cl

    def pubkey_hash(self, fmt: int, x: int, y: int) -> bytes:
        out = ctypes.create_string_buffer(32)
        self.L.hdh_pubkey_hash(fmt, b32(x), b32(y), out)
        return out.raw

    def verify(self, batch, admitted_sorted: np.ndarray, compressed: bool = True):
        n = len(batch)
        ver = np.zeros(n, np.uint8)
        rec = np.zeros((n, 32), np.uint8)
        sgn = np.zeros(n, np.int32)
        adm = np.ascontiguousarray(admitted_sorted, dtype=np.uint8).reshape(-1, 32)
        self.L.hdh_verify(n, _p(batch.type), _p(batch.height), _p(batch.round), _p(batch.valid_round),
                          _p(batch.value), _p(batch.frm), _p(batch.sig), _p(adm), len(adm), int(compressed),
                          _p(ver), _p(rec), _p(sgn))
        return ver, rec, sgn
