"""CPU restatement of hyperdrive's message wire encoding (surge), for arrays.

TEST INFRASTRUCTURE ONLY: imported by tests/ (and bench.py's checks) as the
checker of include/hd_codec.h; the product never imports it.

Restates process/message.go:
  Propose.Marshal / Unmarshal    :102-149   Height, Round, ValidRound, Value, From
  Prevote.Marshal / Unmarshal    :208-247   Height, Round, Value, From
  Precommit.Marshal / Unmarshal  :306-345   Height, Round, Value, From
with renproject/surge v1.2.5's encodings (go.mod:10): int64 -> 8 bytes big
endian two's complement, [32]byte -> 32 raw bytes, no prefixes.  (Parity of
the surge byte order is "unpinned" in this container)
A signed record appends the 65-byte id.Signature raw (the surge encoding of
a {message, [65]byte} struct).
"""
from __future__ import annotations

import struct
from typing import List, Optional, Tuple

PROPOSE, PREVOTE, PRECOMMIT = 1, 2, 3
M64 = (1 << 64) - 1


def record_size(mtype: int, with_sig: bool) -> int:
    if mtype not in (PROPOSE, PREVOTE, PRECOMMIT):
        return 0
    return (88 if mtype == PROPOSE else 80) + (65 if with_sig else 0)


def _be64(x: int) -> bytes:
    return struct.pack(">Q", x & M64)


def _sbe64(b: bytes) -> int:
    v = struct.unpack(">Q", b)[0]
    return v - (1 << 64) if v >> 63 else v


def marshal(mtype: int, height: int, round_: int, valid_round: int, value: bytes, frm: bytes,
            sig: Optional[bytes] = None) -> bytes:
    """One message (message.go:102-124 / 208-226 / 306-324), then the signature."""
    assert len(value) == 32 and len(frm) == 32
    out = _be64(height) + _be64(round_)
    if mtype == PROPOSE:
        out += _be64(valid_round)
    out += value + frm
    if sig is not None:
        assert len(sig) == 65
        out += sig
    return out


def unmarshal(mtype: int, buf: bytes, with_sig: bool):
    """One record -> (height, round, valid_round, value, from, sig) or None when
    the buffer is too short (message.go:126-149 returns "unexpected end")."""
    n = record_size(mtype, with_sig)
    if len(buf) < n:
        return None
    h, r = _sbe64(buf[0:8]), _sbe64(buf[8:16])
    off = 16
    vr = -1
    if mtype == PROPOSE:
        vr = _sbe64(buf[16:24])
        off = 24
    value, frm = buf[off:off + 32], buf[off + 32:off + 64]
    sig = buf[off + 64:off + 129] if with_sig else None
    return h, r, vr, value, frm, sig


def marshal_array(mtype: int, heights, rounds, valid_rounds, values, froms, sigs=None) -> bytes:
    return b"".join(marshal(mtype, int(heights[i]), int(rounds[i]),
                            int(valid_rounds[i]) if valid_rounds is not None else -1,
                            bytes(values[i]), bytes(froms[i]), bytes(sigs[i]) if sigs is not None else None)
                    for i in range(len(heights)))


def unmarshal_array(mtype: int, buf: bytes, n: int, with_sig: bool) -> List[Optional[Tuple]]:
    s = record_size(mtype, with_sig)
    return [unmarshal(mtype, buf[i * s:(i + 1) * s], with_sig) for i in range(n)]
