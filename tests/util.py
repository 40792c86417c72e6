"""Test helpers: oracle-batch conversion and an OpenSSL (libcrypto 3) secp256k1
ECDSA verifier used as an implementation-independent cross-check."""
from __future__ import annotations

import ctypes
import ctypes.util

import numpy as np


def to_np(ob):
    """oracle Batch (lists) -> hyperdrive_amd.verify.Batch (numpy SoA)."""
    from hyperdrive_amd.verify import Batch
    return Batch.from_lists(ob.mtype, ob.height, ob.round, ob.valid_round, ob.value, ob.frm, ob.sig)


def from_np(b):
    import hd_pyoracle as O
    ob = O.Batch()
    vr = b.valid_round if b.valid_round is not None else np.full(len(b), -1, np.int64)
    for i in range(len(b)):
        ob.append(int(b.type[i]), int(b.height[i]), int(b.round[i]), int(vr[i]), b.value[i].tobytes(),
                  b.frm[i].tobytes(), b.sig[i].tobytes())
    return ob


class OpenSSL:
    """secp256k1 via OpenSSL's (deprecated but shipped) EC_KEY/ECDSA API."""
    NID_secp256k1 = 714

    def __init__(self):
        path = ctypes.util.find_library("crypto")
        if not path:
            raise RuntimeError("libcrypto not found")
        L = ctypes.CDLL(path)
        self.L = L
        vp = ctypes.c_void_p
        for name, res, args in [
            ("EC_KEY_new_by_curve_name", vp, [ctypes.c_int]),
            ("EC_KEY_get0_group", vp, [vp]),
            ("EC_KEY_set_public_key", ctypes.c_int, [vp, vp]),
            ("EC_KEY_free", None, [vp]),
            ("EC_POINT_new", vp, [vp]),
            ("EC_POINT_free", None, [vp]),
            ("EC_POINT_oct2point", ctypes.c_int, [vp, vp, ctypes.c_char_p, ctypes.c_size_t, vp]),
            ("EC_POINT_point2oct", ctypes.c_size_t, [vp, vp, ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t, vp]),
            ("EC_POINT_mul", ctypes.c_int, [vp, vp, vp, vp, vp, vp]),
            ("BN_bin2bn", vp, [ctypes.c_char_p, ctypes.c_int, vp]),
            ("BN_free", None, [vp]),
            ("ECDSA_SIG_new", vp, []),
            ("ECDSA_SIG_set0", ctypes.c_int, [vp, vp, vp]),
            ("ECDSA_SIG_free", None, [vp]),
            ("ECDSA_do_verify", ctypes.c_int, [ctypes.c_char_p, ctypes.c_int, vp, vp]),
        ]:
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        self.key = L.EC_KEY_new_by_curve_name(self.NID_secp256k1)
        self.group = L.EC_KEY_get0_group(self.key)

    def verify(self, digest: bytes, r: int, s: int, pub65: bytes) -> bool:
        L = self.L
        pt = L.EC_POINT_new(self.group)
        try:
            if L.EC_POINT_oct2point(self.group, pt, pub65, len(pub65), None) != 1:
                return False
            if L.EC_KEY_set_public_key(self.key, pt) != 1:
                return False
            sig = L.ECDSA_SIG_new()
            L.ECDSA_SIG_set0(sig, L.BN_bin2bn(r.to_bytes(32, "big"), 32, None),
                             L.BN_bin2bn(s.to_bytes(32, "big"), 32, None))
            ok = L.ECDSA_do_verify(digest, len(digest), sig, self.key)
            L.ECDSA_SIG_free(sig)
            return ok == 1
        finally:
            L.EC_POINT_free(pt)

    def pubkey(self, sk: int, compressed: bool = False) -> bytes:
        L = self.L
        pt = L.EC_POINT_new(self.group)
        bn = L.BN_bin2bn(sk.to_bytes(32, "big"), 32, None)
        try:
            assert L.EC_POINT_mul(self.group, pt, bn, None, None, None) == 1
            buf = ctypes.create_string_buffer(65)
            form = 2 if compressed else 4  # POINT_CONVERSION_COMPRESSED / UNCOMPRESSED
            n = L.EC_POINT_point2oct(self.group, pt, form, buf, 65, None)
            return buf.raw[:n]
        finally:
            L.BN_free(bn)
            L.EC_POINT_free(pt)
