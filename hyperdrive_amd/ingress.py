"""Batch ingress of one replica on the GPU: wire bytes -> SoA -> verify ->
message queue -> the current height's vote logs.

The reference handles one message per channel receive (replica/replica.go:
88-151): authentication is the caller's job, ``filterHeight`` drops heights
below the Process's (:247-249), ``mq.Insert*`` buffers per sender
(mq/mq.go:85-143), and ``flush`` consumes the current height into
``process.Propose/Prevote/Precommit`` (:253-265), whose vote logs the count
rules read (process/process.go:823-892).  ``Ingress`` runs the same chain
for a whole batch:

    ing = Ingress(verifier, height=h)
    ing.push_wire(PREVOTE, buf, n)          # unmarshal + verify + filterHeight + mq insert (GPU)
    res = ing.flush()                       # mq.Consume(h, procsAllowed) + vote-log inserts (host table)
    res.proposes                            # handed to the CPU's insertPropose (scheduler/validator)
    res.events                              # HD_VOTE_EV_* quorum crossings per delivered vote (f known)
    ing.advance_height(h + 1)               # the Process committed: CurrentHeight++, logs emptied (process.go:710-725)
    ing.reset_height(h + 5, signatories)    # ResetHeight: ignored unless above the current height
                                            # (replica.go:222-225); logs emptied, mq.DropMessagesBelowHeight,
                                            # a new signatory set rebuilds procsAllowed and f (replica.go:132-145)

Membership follows the reference: every *authenticated* message
(recovered signatory == From: verdict VALID or NOT_ADMITTED) with height >=
the current height is buffered, in the queue of its From; procsAllowed -- the
verifier's admitted set at flush time -- is applied when the queue is
consumed (mq/mq.go:49-51).  A message buffered while its sender was not
admitted is delivered after a reset_height that admits it.

Batch semantics: a flush consumes everything buffered at the current height
in one go; the reference may advance the height in the middle of a flush
(a commit inside process.Precommit), which the caller reproduces by calling
``reset_height`` and flushing again.
"""
from __future__ import annotations

from typing import Optional

import numpy as np

from .codec import record_size, unmarshal_device
from .device import DeviceBatch, _torch, verify_streams, work_stream
from .mq import MessageQueue
from .verify import PROPOSE, Batch, Verifier
from .votes import VoteLog


class FlushResult:
    """One flush's delivery.  consumed: every message delivered (sender in
    procsAllowed), in consumption order; senders: int32 sender-queue id per
    delivered message (queue creation order); vote_status: HD_VOTE_* per
    consumed message (NOT_VOTE for proposes); double_of: batch index of the
    logged vote for DOUBLE, else votes.NO_INDEX; proposes: indices (into
    consumed) of the proposes, for the CPU (computed on first access);
    removed: messages consumed, delivered or dropped by procsAllowed
    (Consume's n); events: uint8 HD_VOTE_EV_* per consumed message
    (votes.EV_*), f known.  (A plain slotted class: a flush per height builds
    one, and a dataclass's init showed in the per-flush host time.)"""
    __slots__ = ("consumed", "senders", "vote_status", "double_of", "removed", "events", "_proposes")

    def __init__(self, consumed: Batch, senders: np.ndarray, vote_status: np.ndarray, double_of: np.ndarray,
                 proposes: Optional[np.ndarray] = None, removed: int = 0, events: Optional[np.ndarray] = None):
        self.consumed = consumed
        self.senders = senders
        self.vote_status = vote_status
        self.double_of = double_of
        self._proposes = proposes
        self.removed = removed
        self.events = events

    @property
    def proposes(self) -> np.ndarray:
        if self._proposes is None:
            self._proposes = np.flatnonzero(self.consumed.type == PROPOSE)
        return self._proposes


class PendingPush:
    """push_wires_begin's handle: the combined device batch, its verdict
    tensor (being written), the rows used, the verify streams and the
    per-buffer verdict views."""
    __slots__ = ("every", "verdicts", "lo", "used", "out")

    def __init__(self, every, verdicts, lo, used, out):
        self.every, self.verdicts, self.lo, self.used, self.out = every, verdicts, lo, used, out


class Ingress:
    def __init__(self, v: Verifier, height: int = 1, max_capacity: int = 1000):
        self.v = v
        self.height = int(height)
        self.mq = MessageQueue(v, max_capacity)
        self.votes = VoteLog(self.height)
        # f = len(signatories) / 3 (replica.go:54, 138): from the verifier's
        # admitted set now, and again on every ResetHeight with a new set; the
        # vote logs report the 2f+1 / f+1 crossings with it
        self.f = None
        if getattr(v, "n_signatories", 0):
            self._set_f(v.n_signatories // 3)
        # (height, insert count) of the last consume: while the queue has had
        # no insert since, every message in it is above that height, so a
        # ResetHeight to at most height + 1 has nothing to drop
        self._clean = None

    def _set_f(self, f: int) -> None:
        self.f = int(f)
        self.votes.set_f(self.f)

    def close(self):
        self.mq.close()
        self.votes.close()

    def push_device(self, batch: DeviceBatch, stream=None):
        """Authenticate a device batch and buffer its authenticated messages
        (VALID or NOT_ADMITTED) with height >= the current height.  Returns
        the device verdict tensor (authenticate_batch_device's: a message
        that fails its From's known-key check is NOT_AUTHENTIC, unclassified)."""
        torch = _torch()
        dev = batch.height.device
        n = batch.n
        verdict = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
        if n == 0:
            return verdict[:0]
        ws = stream or work_stream(dev)
        ws.wait_stream(torch.cuda.current_stream(ws.device))
        self.v.authenticate_batch_device(batch.c_struct(), verdict.data_ptr(), ws.cuda_stream)
        self.mq.insert_verified_device(batch, verdict, self.height, stream=ws)
        return verdict[:n]

    def push_wire(self, mtype: int, buf, n: int, with_sig: bool = True, stream=None):
        """Unmarshal n `mtype` records from a device byte buffer and push them.
        Records the buffer ends inside are dropped (Unmarshal's error,
        process/message.go:126-149).  Returns the verdicts of the complete records."""
        size = record_size(mtype, with_sig)
        complete = min(n, buf.numel() // size) if size else 0
        if complete == 0:
            return _torch().empty(0, dtype=_torch().uint8, device=buf.device)
        db, _ = unmarshal_device(self.v, mtype, buf, complete, with_sig, stream=stream)
        return self.push_device(db, stream=stream)

    def push_wires(self, parts, with_sig: bool = True):
        """Several wire buffers [(mtype, device byte buffer, n), ...] in
        arrival order.  Each is unmarshalled into its rows of one combined
        device batch and verified on one of two streams, alternating, so the
        buffers' verify calls run concurrently on the device (one call's
        fallback recoveries and inversion kernels leave most SIMD slots to the
        other's); the combined batch then goes into the mq with ONE insert
        (arrival order is batch order: inserting the buffers one after another
        keeps the same messages, hd_mq.h -- each insert re-sorts the whole
        queue, so one insert instead of two saves a full sort and its host
        round trips).  Returns the verdicts of each buffer's complete records.
        = push_finish(push_wires_begin(parts))."""
        return self.push_finish(self.push_wires_begin(parts, with_sig))

    def push_wires_begin(self, parts, with_sig: bool = True) -> "PendingPush":
        """The device half of push_wires: the unmarshal and authentication of
        every buffer are queued on the verify streams and the call returns
        without waiting.  The queue is untouched until push_finish, so the
        caller may flush (serve the current heights from the queue, the
        replica's flush, replica.go:251-264) while these messages are being
        authenticated: the reference's loop handles a message only after the
        ones before it (replica.go:100-147), and messages still in
        authentication have not reached the replica yet.  filterHeight
        (replica.go:247-249) applies at push_finish, with the height then."""
        torch = _torch()
        if not parts:
            return PendingPush(None, None, 0, [], [])
        dev = parts[0][1].device
        if getattr(self, "_streams", None) is None or self._streams[0].device != dev:
            self._streams = verify_streams(dev, 2)
        # every stream waits for the caller's work queued so far (the wire
        # buffers), not for each other: with the caller's stream being one of
        # the two, waiting on "the current stream" inside the loop would chain
        # each buffer's verification behind the previous one's
        sizes = []
        for mtype, buf, n in parts:
            size = record_size(mtype, with_sig)
            sizes.append(min(n, buf.numel() // size) if size else 0)
        # each buffer's rows start at a multiple of 16 (unmarshal_device's
        # 16-byte aligned sig rows); the rows between buffers keep verdict 0xFF,
        # which the insert skips
        total = sum((c + 15) // 16 * 16 for c in sizes)
        every = DeviceBatch.empty(max(total, 1), str(dev))
        verdicts = torch.full((max(total, 1),), 0xFF, dtype=torch.uint8, device=dev)
        ready = torch.cuda.Event()   # after the fill above, on the same (current) stream
        ready.record(torch.cuda.current_stream(dev))
        out, used, lo = [], [], 0
        for k, ((mtype, buf, _), complete) in enumerate(zip(parts, sizes)):
            if complete == 0:
                out.append(torch.empty(0, dtype=torch.uint8, device=dev))
                continue
            s = self._streams[k % 2]
            s.wait_event(ready)
            rows = every.rows(lo, complete)
            db, _ = unmarshal_device(self.v, mtype, buf, complete, with_sig, stream=s, sync=False, out=rows,
                                     wait=False)
            verdict = verdicts[lo: lo + complete]
            self.v.authenticate_batch_device(db.c_struct(), verdict.data_ptr(), s.cuda_stream)
            out.append(verdict)
            used.append(s)
            lo += (complete + 15) // 16 * 16
        return PendingPush(every, verdicts, lo, used, out)

    def push_finish(self, pend: "PendingPush"):
        """The queue half of push_wires: filterHeight at the current height
        and the one mq insert of the authenticated messages (after their
        verification, in stream order).  Returns the verdicts of each
        buffer's complete records."""
        if pend.used:
            s0 = pend.used[0]
            for s in pend.used[1:]:
                if s is not s0:
                    s0.wait_stream(s)
            self.mq.insert_verified_device(pend.every.rows(0, pend.lo), pend.verdicts[:pend.lo], self.height,
                                           stream=s0)
        return pend.out

    def flush(self) -> FlushResult:
        """mq.Consume(CurrentHeight, ..., procsAllowed) with procsAllowed = the
        verifier's admitted set now, then the vote-log inserts."""
        mq = self.mq
        b, senders, status, double_of, events = mq.consume_votes(self.height, self.votes)
        self.votes.last_events = events
        self._clean = (self.height, mq.inserts)
        return FlushResult(b, senders, status, double_of, None, mq.last_removed, events)

    def advance_height(self, height: int) -> None:
        """The Process's own height change after a commit (process.go:710-725:
        CurrentHeight = height, vote logs emptied); the queue keeps its
        messages (Consume removes every message at or below the height it
        consumes, mq.go:36-66)."""
        if int(height) <= self.height:
            raise ValueError(f"advance_height({height}) at height {self.height}")
        self.height = int(height)
        self.votes.reset(self.height)

    def reset_height(self, height: int, signatories=None) -> bool:
        """Replica.ResetHeight (replica.go:216-235): ignored (returns False)
        unless `height` is above the current height (:223-225).  Otherwise the
        ResetHeightMessage (:132-145): the logs restart at `height`, lower
        heights leave the queue, and a non-empty signatory set replaces
        procsAllowed (the verifier's admitted set) and f."""
        if int(height) <= self.height:
            return False
        self.height = int(height)
        self.votes.reset(self.height)
        clean = self._clean is not None and self._clean[1] == self.mq.inserts and self.height <= self._clean[0] + 1
        if not clean:
            self.mq.drop_below(self.height)
        if signatories is not None and len(signatories):
            self.v.set_signatories(signatories)
            self._set_f(len(signatories) // 3)
        return True


__all__ = ["Ingress", "FlushResult", "PendingPush"]
