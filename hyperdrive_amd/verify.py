"""Host-side mirror of the batch-verify boundary.

In the reference the authentication of a Propose/Prevote/Precommit is a
precondition the caller must establish before ``Replica.Propose/Prevote/
Precommit`` (replica/replica.go:153-181; mq/mq.go:85-101 "assumes that the
sender has already been authenticated"), and membership is the
``procsAllowed`` filter at consume time (mq/mq.go:49-51).  This module is the
Python face of the C ABI that takes over both for a whole batch:

    v = Verifier(device=0)
    v.set_signatories(signatories)          # replica.go:69-72 / 136-144
    res = v.verify_batch(batch)             # per-message verdicts
    t = v.tally(batch, res.verdict)         # first-wins logs + 2f+1 counts

Per-message failures are verdicts (never exceptions); exceptions are raised
only for invalid arguments and device failures, like the reference's
``fmt.Errorf`` returns in process/message.go:61-77.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Dict, Optional, Sequence, Tuple

import numpy as np

from . import _lib
from ._lib import HDError, HdBatch, HdTallyOut

# verdicts (include/hd_verify.h)
VALID = 0
BAD_RECID = 1
BAD_RS = 2
NO_POINT = 3
INFINITY = 4
SIGNATORY_MISMATCH = 5
NOT_ADMITTED = 6
BAD_TYPE = 7
NOT_AUTHENTIC = 8     # authenticate_batch_device only (include/hd_verify.h)
VERDICT_NAMES = ["VALID", "BAD_RECID", "BAD_RS", "NO_POINT", "INFINITY", "SIGNATORY_MISMATCH",
                 "NOT_ADMITTED", "BAD_TYPE", "NOT_AUTHENTIC"]

PROPOSE, PREVOTE, PRECOMMIT = 1, 2, 3


def _ptr(a: Optional[np.ndarray]):
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"], "arrays must be C-contiguous"
    return a.ctypes.data


@dataclass
class Batch:
    """Structure-of-arrays batch in host memory (hd_batch)."""
    type: np.ndarray          # uint8[n]
    height: np.ndarray        # int64[n]
    round: np.ndarray         # int64[n]
    valid_round: Optional[np.ndarray]  # int64[n] or None
    value: np.ndarray         # uint8[n, 32]
    frm: np.ndarray           # uint8[n, 32]
    sig: np.ndarray           # uint8[n, 65]

    def __post_init__(self):
        n = len(self.type)
        self.type = np.ascontiguousarray(self.type, dtype=np.uint8)
        self.height = np.ascontiguousarray(self.height, dtype=np.int64)
        self.round = np.ascontiguousarray(self.round, dtype=np.int64)
        if self.valid_round is not None:
            self.valid_round = np.ascontiguousarray(self.valid_round, dtype=np.int64)
        self.value = np.ascontiguousarray(self.value, dtype=np.uint8).reshape(n, 32)
        self.frm = np.ascontiguousarray(self.frm, dtype=np.uint8).reshape(n, 32)
        self.sig = np.ascontiguousarray(self.sig, dtype=np.uint8).reshape(n, 65)
        for name in ("height", "round"):
            if len(getattr(self, name)) != n:
                raise ValueError(f"{name} has {len(getattr(self, name))} entries, expected {n}")
        if self.valid_round is not None and len(self.valid_round) != n:
            raise ValueError("valid_round length mismatch")

    def __len__(self) -> int:
        return len(self.type)

    @classmethod
    def _wrap(cls, mtype, height, round_, valid_round, value, frm, sig) -> "Batch":
        """Fields the library just wrote (contiguous, right dtypes and shapes):
        no conversion pass (the per-flush result of the mq consume)."""
        b = object.__new__(cls)
        b.type, b.height, b.round, b.valid_round, b.value, b.frm, b.sig = (mtype, height, round_, valid_round, value,
                                                                           frm, sig)
        return b

    @classmethod
    def from_lists(cls, mtype, height, round_, valid_round, value, frm, sig) -> "Batch":
        n = len(mtype)
        return cls(np.array(mtype, np.uint8), np.array(height, np.int64), np.array(round_, np.int64),
                   np.array(valid_round, np.int64) if valid_round is not None else None,
                   np.frombuffer(b"".join(value), np.uint8).reshape(n, 32).copy() if n else np.zeros((0, 32), np.uint8),
                   np.frombuffer(b"".join(frm), np.uint8).reshape(n, 32).copy() if n else np.zeros((0, 32), np.uint8),
                   np.frombuffer(b"".join(sig), np.uint8).reshape(n, 65).copy() if n else np.zeros((0, 65), np.uint8))

    def c_struct(self) -> HdBatch:
        return HdBatch(len(self), _ptr(self.type), _ptr(self.height), _ptr(self.round), _ptr(self.valid_round),
                       _ptr(self.value), _ptr(self.frm), _ptr(self.sig))


@dataclass
class CompactBatch:
    """The PCIe-lean host batch (hd_batch_compact): From and value as 16-bit
    indices into the signatory array of the context (then escape rows) and
    into a per-batch value dictionary."""
    type: np.ndarray          # uint8[n]
    height: np.ndarray        # int64[n]
    round: np.ndarray         # int64[n]
    valid_round: Optional[np.ndarray]
    from_idx: np.ndarray      # uint16[n]
    value_idx: np.ndarray     # uint16[n]
    sig: np.ndarray           # uint8[n, 65]
    escape: np.ndarray        # uint8[n_escape, 32]
    values: np.ndarray        # uint8[n_values, 32]

    def __len__(self):
        return len(self.type)

    @staticmethod
    def from_batch(b: "Batch", signatories) -> "CompactBatch":
        """Index form of a Batch against the signatory array the context was
        given (the first row of a repeated signatory is used; Froms outside
        it become escape rows, values the batch's dictionary)."""
        sig = np.ascontiguousarray(_as_rows(signatories, 32))
        n, ns = len(b), len(sig)
        key = lambda rows: rows.view(np.dtype((np.void, 32))).ravel()
        skeys = key(sig)
        order = np.argsort(skeys, kind="stable")
        fk = key(b.frm)
        pos = np.searchsorted(skeys[order], fk)
        pos = np.minimum(pos, max(ns - 1, 0))
        hit = (skeys[order][pos] == fk) if ns else np.zeros(n, bool)
        from_idx = np.zeros(n, np.int64)
        from_idx[hit] = order[pos[hit]]
        esc_rows, esc_inv = np.unique(fk[~hit], return_inverse=True)
        from_idx[~hit] = ns + esc_inv.ravel()
        vals, vinv = np.unique(key(b.value), return_inverse=True)
        if ns + len(esc_rows) > 65536 or len(vals) > 65536:
            raise ValueError("more than 65536 From rows or values: split the batch")
        return CompactBatch(b.type, b.height, b.round, b.valid_round, from_idx.astype(np.uint16),
                            vinv.ravel().astype(np.uint16), b.sig,
                            np.frombuffer(esc_rows.tobytes(), np.uint8).reshape(-1, 32).copy(),
                            np.frombuffer(vals.tobytes(), np.uint8).reshape(-1, 32).copy())

    def c_struct(self):
        from ._lib import HdBatchCompact
        return HdBatchCompact(len(self), _ptr(self.type), _ptr(self.height), _ptr(self.round), _ptr(self.valid_round),
                              _ptr(self.from_idx), _ptr(self.value_idx), _ptr(self.sig), len(self.escape),
                              _ptr(self.escape) if len(self.escape) else None, len(self.values), _ptr(self.values))


@dataclass
class VerifyResult:
    verdict: np.ndarray       # uint8[n]
    recovered: np.ndarray     # uint8[n, 32]
    valid_bitmap: np.ndarray  # uint32[ceil(n/32)]


@dataclass
class TallyResult:
    """First-wins vote logs summarised per (h, r) and per (h, r, type, value)."""
    count: Dict[Tuple[int, int, int, bytes], int]
    distinct: Dict[Tuple[int, int, int], int]
    distinct_any: Dict[Tuple[int, int], int]
    dup: np.ndarray           # uint8[n]: 0 logged, 1 identical dup, 2 double vote, 3 not a candidate


class Verifier:
    """One context per caller thread (the reference's Process is
    single-goroutine, process/process.go:100-101)."""

    def __init__(self, device: int = 0, compressed=True):
        """compressed: the pubkey encoding of id.NewSignatory -- True / 1 SEC1
        compressed (33 B, default), False / 0 SEC1 uncompressed (65 B),
        2 raw X || Y (64 B), 3 X.Bytes() || Y.Bytes() (Go minimal encodings,
        <= 64 B) (include/hd_verify.h HD_PUBKEY_*)."""
        self._lib = _lib.load()
        h = ctypes.c_void_p()
        rc = self._lib.hd_ctx_create(device, ctypes.byref(h))
        if rc != 0:
            raise HDError(rc, "hd_ctx_create")
        self._ctx = h
        self._close_rank = 1          # closed after the queues / tables that use it
        _lib.track(self)
        self.device = device
        self._check(self._lib.hd_ctx_set_pubkey_format(self._ctx, int(compressed)), "set_pubkey_format")
        self.n_signatories = 0

    def _check(self, rc: int, where: str):
        if rc != 0:
            detail = self._lib.hd_ctx_last_error(self._ctx).decode() if self._ctx else ""
            raise HDError(rc, where, detail)

    def close(self):
        if getattr(self, "_ctx", None):
            self._lib.hd_ctx_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @property
    def handle(self):
        return self._ctx

    def set_signatories(self, signatories) -> None:
        arr = _as_rows(signatories, 32)
        self._check(self._lib.hd_set_signatories(self._ctx, _ptr(arr), len(arr)), "hd_set_signatories")
        self.n_signatories = len(arr)

    # include/hd_verify.h HD_VAR_*: kernel variants of this context
    VARIANTS = {"verify_waves": 0, "sum_waves": 1, "sum_prefetch": 2, "split_k": 4, "recover_g": 5,
                "key_width": 7, "wave_prio": 8, "foreign_keys": 10, "slow_lift": 11}

    def set_variant(self, name: str, value: int) -> None:
        """Select a compiled kernel variant (A/B, variant tests); see
        include/hd_verify.h HD_VAR_* for the keys and values."""
        self._check(self._lib.hd_ctx_set_variant(self._ctx, self.VARIANTS[name], int(value)), "hd_ctx_set_variant")

    def variant(self, name: str) -> int:
        v = ctypes.c_int()
        self._check(self._lib.hd_ctx_get_variant(self._ctx, self.VARIANTS[name], ctypes.byref(v)), "hd_ctx_get_variant")
        return v.value

    def set_fastpath(self, enable: bool) -> None:
        """Known-key fast path on/off (include/hd_verify.h hd_ctx_set_fastpath)."""
        self._check(self._lib.hd_ctx_set_fastpath(self._ctx, 1 if enable else 0), "hd_ctx_set_fastpath")

    def profile(self, enable: bool) -> None:
        """Record HIP events around every verify call and its k_fast_sums
        launch (include/hd_verify.h hd_ctx_profile)."""
        self._check(self._lib.hd_ctx_profile(self._ctx, 1 if enable else 0), "hd_ctx_profile")

    def profile_read(self):
        """(calls, verify ms summed, k_fast_sums launches, their ms summed)
        since the last read."""
        c, s = ctypes.c_uint32(), ctypes.c_uint32()
        vm, sm = ctypes.c_double(), ctypes.c_double()
        self._check(self._lib.hd_ctx_profile_read(self._ctx, ctypes.byref(c), ctypes.byref(vm), ctypes.byref(s),
                                                  ctypes.byref(sm)), "hd_ctx_profile_read")
        return c.value, vm.value, s.value, sm.value

    def fastpath_stats(self) -> Tuple[int, int]:
        """(signatories with built key tables, messages of the last verify
        call that took the full recovery)."""
        k, f = ctypes.c_uint32(), ctypes.c_uint32()
        self._check(self._lib.hd_ctx_fastpath_stats(self._ctx, ctypes.byref(k), ctypes.byref(f)),
                    "hd_ctx_fastpath_stats")
        return int(k.value), int(f.value)

    def foreign_stats(self, checks: bool = False):
        """(foreign-key slots with built tables, slotless Froms promoted so far
        into a colder foreign key's slot[, eviction checks so far])."""
        r, e, c = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        self._check(self._lib.hd_ctx_foreign_stats(self._ctx, ctypes.byref(r), ctypes.byref(e), ctypes.byref(c)),
                    "hd_ctx_foreign_stats")
        return (int(r.value), int(e.value), int(c.value)) if checks else (int(r.value), int(e.value))

    def fastpath_geometry(self) -> Tuple[int, int, int]:
        """(G table windows, per-key table windows, messages sharing one
        inversion) of the known-key check as this context runs it."""
        g, k, m = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        self._check(self._lib.hd_ctx_fastpath_geometry(self._ctx, ctypes.byref(g), ctypes.byref(k), ctypes.byref(m)),
                    "hd_ctx_fastpath_geometry")
        return int(g.value), int(k.value), int(m.value)

    def known_keys(self) -> int:
        return self.fastpath_stats()[0]

    def verify_batch(self, batch: Batch, recovered: bool = True) -> VerifyResult:
        n = len(batch)
        verdict = np.zeros(n, np.uint8)
        rec = np.zeros((n, 32), np.uint8)
        bitmap = np.zeros((n + 31) // 32, np.uint32)
        cb = batch.c_struct()
        self._check(self._lib.hd_verify_batch(self._ctx, ctypes.byref(cb), _ptr(verdict),
                                              _ptr(rec) if recovered else None, _ptr(bitmap)), "hd_verify_batch")
        return VerifyResult(verdict, rec, bitmap)

    def submit(self, batch: Batch, verdict: np.ndarray, recovered: Optional[np.ndarray] = None,
               bitmap: Optional[np.ndarray] = None) -> int:
        """Asynchronous host-buffer verification (hd_verify_submit): returns a
        ticket; the outputs land in the given arrays by wait(ticket).  The
        batch arrays and the outputs must stay alive (and the inputs
        unchanged) until then; pinned arrays (torch pin_memory / pinned_empty)
        move by DMA without a staging copy."""
        cb = batch.c_struct()
        t = ctypes.c_uint64()
        self._check(self._lib.hd_verify_submit(self._ctx, ctypes.byref(cb), _ptr(verdict), _ptr(recovered),
                                               _ptr(bitmap), ctypes.byref(t)), "hd_verify_submit")
        return t.value

    def submit_compact(self, batch: CompactBatch, verdict: np.ndarray, recovered: Optional[np.ndarray] = None,
                       bitmap: Optional[np.ndarray] = None) -> int:
        """hd_verify_submit_compact: as submit, with From and value as indices
        (CompactBatch.from_batch); the outputs are the expanded batch's."""
        cb = batch.c_struct()
        t = ctypes.c_uint64()
        self._check(self._lib.hd_verify_submit_compact(self._ctx, ctypes.byref(cb), _ptr(verdict), _ptr(recovered),
                                                       _ptr(bitmap), ctypes.byref(t)), "hd_verify_submit_compact")
        return t.value

    def wait(self, ticket: int) -> None:
        self._check(self._lib.hd_verify_wait(self._ctx, int(ticket)), "hd_verify_wait")

    def verify_batch_device(self, dbatch: HdBatch, d_verdict: int, d_recovered: Optional[int] = None,
                            d_signer: Optional[int] = None, d_bitmap: Optional[int] = None,
                            stream: Optional[int] = None) -> None:
        """Device-resident variant: every pointer is a device address."""
        self._check(self._lib.hd_verify_batch_device(self._ctx, ctypes.byref(dbatch), d_verdict, d_recovered,
                                                     d_signer, d_bitmap, stream), "hd_verify_batch_device")

    def authenticate_batch_device(self, dbatch: HdBatch, d_verdict: int, stream: Optional[int] = None) -> None:
        """Verdicts for the replica ingress (hd_authenticate_batch_device):
        VALID and NOT_ADMITTED exactly as verify_batch_device; a message whose
        From has a known key that does not verify its signature is final as
        NOT_AUTHENTIC, without the recovery that would classify it (the
        reference drops every unauthenticated message, process/process.go:95-98)."""
        self._check(self._lib.hd_authenticate_batch_device(self._ctx, ctypes.byref(dbatch), d_verdict, stream),
                    "hd_authenticate_batch_device")

    # ---- tally -------------------------------------------------------
    @staticmethod
    def _tally_struct(n: int, pinned: bool = False):
        """Output arrays for n messages.  pinned: page-locked host memory (torch
        pin_memory), so the library's device-to-host copies are plain DMA on
        the tally's stream instead of staged pageable copies."""
        keep = []

        def mk(dtype):
            if not pinned:
                return np.zeros(max(n, 1), dtype)
            import torch
            tdt = {np.int64: torch.int64, np.uint8: torch.uint8, np.uint32: torch.int32}[dtype]
            t = torch.zeros(max(n, 1), dtype=tdt, pin_memory=True)
            keep.append(t)
            return t.numpy().view(dtype)

        arrs = dict(
            count_height=mk(np.int64), count_round=mk(np.int64), count_type=mk(np.uint8), count_rep=mk(np.uint32),
            count_n=mk(np.uint32), hr_height=mk(np.int64), hr_round=mk(np.int64), hr_prevotes=mk(np.uint32),
            hr_precommits=mk(np.uint32), hr_any=mk(np.uint32), dup=mk(np.uint8), hr_rep=mk(np.uint32))
        if keep:
            arrs["_pinned"] = keep
        t = HdTallyOut()
        t.cap_counts = n
        t.cap_hr = n
        for k, a in arrs.items():
            if not k.startswith("_"):
                setattr(t, k, _ptr(a))
        return t, arrs

    @staticmethod
    def _tally_result(batch: Batch, t: HdTallyOut, a) -> TallyResult:
        count = {}
        for k in range(t.n_counts):
            rep = int(a["count_rep"][k])
            count[(int(a["count_height"][k]), int(a["count_round"][k]), int(a["count_type"][k]),
                   batch.value[rep].tobytes())] = int(a["count_n"][k])
        distinct, distinct_any = {}, {}
        for k in range(t.n_hr):
            h, r = int(a["hr_height"][k]), int(a["hr_round"][k])
            if a["hr_prevotes"][k]:
                distinct[(h, r, PREVOTE)] = int(a["hr_prevotes"][k])
            if a["hr_precommits"][k]:
                distinct[(h, r, PRECOMMIT)] = int(a["hr_precommits"][k])
            distinct_any[(h, r)] = int(a["hr_any"][k])
        return TallyResult(count, distinct, distinct_any, a["dup"][: len(batch)].copy())

    def tally(self, batch: Batch, verdict: np.ndarray) -> TallyResult:
        n = len(batch)
        verdict = np.ascontiguousarray(verdict, dtype=np.uint8)
        t, a = self._tally_struct(n)
        cb = batch.c_struct()
        self._check(self._lib.hd_tally(self._ctx, ctypes.byref(cb), _ptr(verdict), ctypes.byref(t)), "hd_tally")
        return self._tally_result(batch, t, a)

    def process_batch(self, batch: Batch) -> Tuple[VerifyResult, TallyResult]:
        n = len(batch)
        verdict = np.zeros(n, np.uint8)
        rec = np.zeros((n, 32), np.uint8)
        bitmap = np.zeros((n + 31) // 32, np.uint32)
        t, a = self._tally_struct(n)
        cb = batch.c_struct()
        self._check(self._lib.hd_process_batch(self._ctx, ctypes.byref(cb), _ptr(verdict), _ptr(rec), _ptr(bitmap),
                                               ctypes.byref(t)), "hd_process_batch")
        return VerifyResult(verdict, rec, bitmap), self._tally_result(batch, t, a)

    # ---- synthetic workload ------------------------------------------
    def gen_keys(self, S: int) -> Tuple[np.ndarray, np.ndarray]:
        sigs = np.zeros((S, 32), np.uint8)
        foreign = np.zeros((16, 32), np.uint8)
        self._check(self._lib.hd_gen_keys(self._ctx, S, _ptr(sigs), _ptr(foreign)), "hd_gen_keys")
        return sigs, foreign


def _as_rows(x, width: int) -> np.ndarray:
    if isinstance(x, np.ndarray):
        arr = np.ascontiguousarray(x, dtype=np.uint8).reshape(-1, width)
    else:
        x = list(x)
        for s in x:
            if len(s) != width:
                raise ValueError(f"expected {width}-byte entries")
        arr = np.frombuffer(b"".join(x), np.uint8).reshape(-1, width).copy() if x else np.zeros((0, width), np.uint8)
    return arr


def probe_valu(device: int = 0, op: int = 1, iters: int = 2000) -> float:
    """Measured lane-ops/s of one VALU instruction class (include/hd_probe.h)."""
    lib = _lib.load()
    out = ctypes.c_double()
    rc = lib.hd_probe_valu(device, op, iters, ctypes.byref(out))
    if rc != 0:
        raise HDError(rc, "hd_probe_valu")
    return out.value
