"""ctypes binding of ``libhdverify.so`` (include/hd_verify.h, include/hd_probe.h).

The library is the product: there is no Python/CPU fallback.  If it is missing
or fails to load, importing the binding raises immediately.
"""
from __future__ import annotations

import atexit
import ctypes
import os
import weakref

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("HD_LIB", os.path.join(HERE, "_lib", "libhdverify.so"))

HD_OK = 0
HD_EINVAL = -1
HD_ENOMEM = -2
HD_EDEVICE = -3
HD_ECAP = -4
HD_EAGAIN = -5

c_u8p = ctypes.POINTER(ctypes.c_uint8)
c_i8p = ctypes.POINTER(ctypes.c_int8)
c_i64p = ctypes.POINTER(ctypes.c_int64)
c_u32p = ctypes.POINTER(ctypes.c_uint32)
c_i32p = ctypes.POINTER(ctypes.c_int32)


class HdBatch(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_uint32),
        ("type", ctypes.c_void_p),
        ("height", ctypes.c_void_p),
        ("round", ctypes.c_void_p),
        ("valid_round", ctypes.c_void_p),
        ("value32", ctypes.c_void_p),
        ("from32", ctypes.c_void_p),
        ("sig65", ctypes.c_void_p),
    ]


class HdBatchCompact(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_uint32),
        ("type", ctypes.c_void_p),
        ("height", ctypes.c_void_p),
        ("round", ctypes.c_void_p),
        ("valid_round", ctypes.c_void_p),
        ("from_idx", ctypes.c_void_p),
        ("value_idx", ctypes.c_void_p),
        ("sig65", ctypes.c_void_p),
        ("n_escape", ctypes.c_uint32),
        ("escape32", ctypes.c_void_p),
        ("n_values", ctypes.c_uint32),
        ("values32", ctypes.c_void_p),
    ]


class HdBatchOut(ctypes.Structure):
    _fields_ = [
        ("type", ctypes.c_void_p),
        ("height", ctypes.c_void_p),
        ("round", ctypes.c_void_p),
        ("valid_round", ctypes.c_void_p),
        ("value32", ctypes.c_void_p),
        ("from32", ctypes.c_void_p),
        ("sig65", ctypes.c_void_p),
        ("adv_class", ctypes.c_void_p),
    ]


class HdTallyOut(ctypes.Structure):
    _fields_ = [
        ("cap_counts", ctypes.c_uint32),
        ("n_counts", ctypes.c_uint32),
        ("count_height", ctypes.c_void_p),
        ("count_round", ctypes.c_void_p),
        ("count_type", ctypes.c_void_p),
        ("count_rep", ctypes.c_void_p),
        ("count_n", ctypes.c_void_p),
        ("cap_hr", ctypes.c_uint32),
        ("n_hr", ctypes.c_uint32),
        ("hr_height", ctypes.c_void_p),
        ("hr_round", ctypes.c_void_p),
        ("hr_prevotes", ctypes.c_void_p),
        ("hr_precommits", ctypes.c_void_p),
        ("hr_any", ctypes.c_void_p),
        ("dup", ctypes.c_void_p),
        ("hr_rep", ctypes.c_void_p),
    ]


class HdTallyTicket(ctypes.Structure):
    """include/hd_verify.h hd_tally_ticket (hd_tally_device_bitmap_async / hd_tally_collect)."""
    _fields_ = [("stage", ctypes.c_void_p), ("stage_cap", ctypes.c_size_t), ("dup", ctypes.c_int),
                ("n", ctypes.c_uint32), ("H", ctypes.c_uint32), ("Cg", ctypes.c_uint32), ("need", ctypes.c_size_t),
                ("done", ctypes.c_void_p)]


# every symbol include/*.h declares, with its ctypes signature
SIGNATURES = {
    "hd_ctx_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    "hd_ctx_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "hd_ctx_set_pubkey_format": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "hd_set_signatories": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32]),
    "hd_ctx_set_fastpath": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "hd_ctx_fastpath_stats": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32),
                                             ctypes.POINTER(ctypes.c_uint32)]),
    "hd_ctx_foreign_stats": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32),
                                            ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32)]),
    "hd_ctx_fastpath_geometry": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int),
                                                ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
    "hd_ctx_profile": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "hd_ctx_set_variant": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]),
    "hd_ctx_get_variant": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]),
    "hd_ctx_profile_read": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32),
                                           ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_uint32),
                                           ctypes.POINTER(ctypes.c_double)]),
    "hd_verify_batch": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(HdBatch), ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.c_void_p]),
    "hd_verify_batch_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(HdBatch), ctypes.c_void_p,
                                              ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "hd_authenticate_batch_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(HdBatch), ctypes.c_void_p,
                                                    ctypes.c_void_p]),
    "hd_verify_submit": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(HdBatch), ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)]),
    "hd_verify_submit_compact": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(HdBatchCompact), ctypes.c_void_p,
                                                ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)]),
    "hd_verify_wait": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64]),
    "hd_host_alloc": (ctypes.c_int, [ctypes.c_size_t, ctypes.POINTER(ctypes.c_void_p)]),
    "hd_host_free": (ctypes.c_int, [ctypes.c_void_p]),
    "hd_stream_create_dedicated": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p)]),
    "hd_stream_destroy": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "hd_tally": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(HdBatch), ctypes.c_void_p,
                                ctypes.POINTER(HdTallyOut)]),
    "hd_tally_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(HdBatch), ctypes.c_void_p,
                                       ctypes.POINTER(HdTallyOut), ctypes.c_void_p]),
    "hd_tally_device_bitmap_part": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(HdBatch), ctypes.c_void_p,
                                                   ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(HdTallyOut),
                                                   ctypes.c_void_p]),
    "hd_tally_partition_of": (ctypes.c_uint32, [ctypes.c_int64, ctypes.c_int64, ctypes.c_uint32]),
    "hd_tally_device_bitmap": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(HdBatch), ctypes.c_void_p,
                                              ctypes.POINTER(HdTallyOut), ctypes.c_void_p]),
    "hd_tally_device_bitmap_async": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(HdBatch), ctypes.c_void_p,
                                                    ctypes.POINTER(HdTallyTicket), ctypes.c_void_p]),
    "hd_tally_collect": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(HdTallyTicket), ctypes.POINTER(HdTallyOut)]),
    "hd_tally_stage_bytes": (ctypes.c_size_t, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int]),
    "hd_tally_ticket_release": (ctypes.c_int, [ctypes.POINTER(HdTallyTicket)]),
    "hd_process_batch": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(HdBatch), ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(HdTallyOut)]),
    "hd_multi_create": (ctypes.c_int, [ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p)]),
    "hd_multi_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "hd_multi_size": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
    "hd_multi_ctx": (ctypes.c_void_p, [ctypes.c_void_p, ctypes.c_int]),
    "hd_multi_set_signatories": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32]),
    "hd_multi_set_pubkey_format": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "hd_multi_verify_batch": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(HdBatch), ctypes.c_void_p,
                                             ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "hd_route_candidates_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(HdBatch), ctypes.c_void_p,
                                                  ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32,
                                                  ctypes.POINTER(ctypes.c_uint32), ctypes.c_void_p]),
    "hd_route_candidates_listed_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(HdBatch), ctypes.c_void_p,
                                                         ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p,
                                                         ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                                         ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32),
                                                         ctypes.c_void_p]),
    "hd_unroute_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                         ctypes.POINTER(HdBatchOut), ctypes.c_void_p, ctypes.c_void_p]),
    "hd_tally_routed_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(HdBatch), ctypes.c_void_p,
                                              ctypes.POINTER(HdTallyOut), ctypes.c_void_p]),
    "hd_gen_keys": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]),
    "hd_gen_batch_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint32,
                                           ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.POINTER(HdBatchOut), ctypes.c_void_p]),
    "hd_strerror": (ctypes.c_char_p, [ctypes.c_int]),
    "hd_ctx_last_error": (ctypes.c_char_p, [ctypes.c_void_p]),
    "hd_abi_version": (ctypes.c_int, []),
    "hd_probe_valu": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_uint32, ctypes.POINTER(ctypes.c_double)]),
    # include/hd_codec.h
    "hd_record_size": (ctypes.c_uint32, [ctypes.c_int, ctypes.c_int]),
    "hd_unmarshal_batch_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                                 ctypes.c_uint64, ctypes.c_uint32, ctypes.POINTER(HdBatchOut),
                                                 ctypes.c_void_p, ctypes.c_void_p]),
    "hd_marshal_batch_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.POINTER(HdBatch),
                                               ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]),
    # include/hd_mq.h
    "hd_mq_create": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.POINTER(ctypes.c_void_p)]),
    "hd_mq_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "hd_mq_insert_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(HdBatch), ctypes.c_void_p,
                                           ctypes.c_void_p]),
    "hd_mq_insert_verified_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(HdBatch), ctypes.c_void_p,
                                                    ctypes.c_int64, ctypes.c_void_p]),
    "hd_mq_size": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)]),
    "hd_mq_senders": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32)]),
    "hd_mq_consume": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_uint32,
                                     ctypes.POINTER(HdBatchOut), ctypes.c_void_p, ctypes.c_uint32,
                                     ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32)]),
    "hd_mq_consume_votes": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                                           ctypes.c_uint32, ctypes.POINTER(HdBatchOut), ctypes.c_void_p,
                                           ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32),
                                           ctypes.POINTER(ctypes.c_uint32), ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32)]),
    "hd_mq_drop_below": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64]),
    # include/hd_digest.h
    "hd_digest_batch_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(HdBatch),
                                              ctypes.c_void_p, ctypes.c_void_p]),
    "hd_hash_bytes_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]),
    "hd_verify_batch_digest_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(HdBatch), ctypes.c_void_p,
                                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                     ctypes.c_void_p, ctypes.c_void_p]),
    # include/hd_votes.h
    "hd_votes_create": (ctypes.c_int, [ctypes.c_int64, ctypes.POINTER(ctypes.c_void_p)]),
    "hd_votes_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "hd_votes_reset": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64]),
    "hd_votes_height": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64)]),
    "hd_votes_set_f": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32]),
    "hd_votes_insert": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint8, ctypes.c_int64, ctypes.c_int64,
                                       ctypes.c_char_p, ctypes.c_char_p, c_u8p, ctypes.c_void_p, c_u8p]),
    "hd_votes_insert_batch": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(HdBatch), ctypes.c_void_p,
                                             ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                             ctypes.POINTER(ctypes.c_uint32)]),
    "hd_votes_trace_propose": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_char_p, c_u8p]),
    "hd_votes_count": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint8, ctypes.c_int64, ctypes.c_char_p,
                                      ctypes.POINTER(ctypes.c_uint32)]),
    "hd_votes_len": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint8, ctypes.c_int64,
                                    ctypes.POINTER(ctypes.c_uint32)]),
    "hd_votes_trace_len": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(ctypes.c_uint32)]),
    "hd_votes_get": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint8, ctypes.c_int64, ctypes.c_char_p,
                                    ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]),
}

_LIB = None


def load(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load libhdverify.so (once) and attach the signatures.  Raises if absent."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(path):
        raise RuntimeError(
            f"hyperdrive_amd native library not found at {path}; build it with "
            "`python -m hyperdrive_amd.build` (there is no CPU fallback)")
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        if "HD_LIB" in os.environ and not hasattr(lib, name):
            continue   # an older build named by HD_LIB (A/B runs): only what it exports
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _LIB = lib
    return lib


class HDError(RuntimeError):
    def __init__(self, code: int, where: str, detail: str = ""):
        lib = load()
        msg = f"{where}: {lib.hd_strerror(code).decode()} ({code})"
        if detail:
            msg += f": {detail}"
        super().__init__(msg)
        self.code = code


# Native handles still open at interpreter exit are closed by an atexit hook
# (queues and vote tables before their contexts), while the HIP runtime and
# torch are still alive, instead of by finalizers during teardown.
_LIVE = weakref.WeakSet()


def track(obj) -> None:
    _LIVE.add(obj)


@atexit.register
def _close_all() -> None:
    for o in sorted(list(_LIVE), key=lambda o: getattr(o, "_close_rank", 0)):
        try:
            o.close()
        except Exception:
            pass
