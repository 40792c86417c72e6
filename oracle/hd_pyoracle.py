"""Pure-Python CPU restatement of hyperdrive's message-authentication + tally path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module, and only as the
checker.  The product path (``hyperdrive_amd``) never imports it.

What it restates (reference = tuanggolt/hyperdrive @ /root/reference, Go):

* digest preimages -- ``process/message.go:53-78`` (NewProposeHash: BE64 h ||
  BE64 r || BE64 validRound || value, 56 B), ``message.go:165-186``
  (NewPrevoteHash) and ``message.go:263-284`` (NewPrecommitHash): BE64 h ||
  BE64 r || value, 48 B, byte-identical for the two vote types (no type tag).
  Encoding = renproject/surge v1.2.5 (go.mod:10): fixed-width big-endian ints,
  ``[32]byte`` raw.  Hash = ``id.NewHash`` = SHA-256 (renproject/id v0.4.2,
  go.mod:9).
* ``id.Signature.Signatory(&hash)`` (call sites ``process/message_test.go:152,
  261, 324``) = go-ethereum v1.9.5 ``crypto.SigToPub`` -> cgo libsecp256k1
  ``secp256k1_ext_ecdsa_recover`` semantics, restated in ``recover()`` below,
  followed by ``id.NewSignatory`` = SHA-256 over the SEC1 *compressed* pubkey
  (33 B; ``compressed=False`` switches to the 65 B uncompressed encoding,
  ``compressed=2`` to the raw 64 B X || Y).
* ``id.PrivKey.Sign`` (``message_test.go:150``) = libsecp256k1
  ``secp256k1_ecdsa_sign_recoverable`` with the RFC6979 HMAC-SHA256 nonce,
  low-S normalisation, V = recid.  Used only to build inputs.
* admitted-set filter ``procsAllowed`` (``replica/replica.go:69-72``) applied
  in ``mq.Consume`` (``mq/mq.go:49-51``).
* first-wins vote logs ``insertPrevote`` / ``insertPrecommit``
  (``process/process.go:823-892``) and the counting loops of the 2f+1 / f+1
  rules (``process.go:486-494, 534, 574-582, 626-632, 658, 696-702, 751``).

Parity anchoring (see DESIGN.md "Oracle"): the reference holds no byte-level
golden vectors for this path; this restatement is pinned by
public known-answer tests (FIPS 180-2 SHA-256 vectors, the secp256k1 generator,
go-ethereum's published ecrecover vector) and cross-checked against OpenSSL's
independent ECDSA verifier in ``tests/test_oracle.py``.
"""
from __future__ import annotations

import hashlib
import hmac
import struct
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

# ---------------------------------------------------------------------------
# curve constants (SEC2 secp256k1)
P = 2**256 - 2**32 - 977
N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
GX = 0x79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798
GY = 0x483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8
M64 = (1 << 64) - 1

# message types -- process/message.go:11-22
PROPOSE, PREVOTE, PRECOMMIT, TIMEOUT = 1, 2, 3, 4

# verdict enum (include/hd_verify.h)
VALID = 0
BAD_RECID = 1
BAD_RS = 2
NO_POINT = 3
INFINITY = 4
SIGNATORY_MISMATCH = 5
NOT_ADMITTED = 6
BAD_TYPE = 7

INVALID_ROUND = -1          # process/state.go:304
NIL_VALUE = bytes(32)       # process/state.go:337


# ---------------------------------------------------------------------------
# digests
def be64(x: int) -> bytes:
    """surge v1.2.5 int64 encoding: 8-byte big-endian two's complement."""
    return struct.pack(">Q", x & M64)


def vote_preimage(height: int, round_: int, value: bytes) -> bytes:
    """NewPrevoteHashWithBuffer / NewPrecommitHashWithBuffer preimage
    (process/message.go:172-186, 270-284)."""
    assert len(value) == 32
    return be64(height) + be64(round_) + value


def propose_preimage(height: int, round_: int, valid_round: int, value: bytes) -> bytes:
    """NewProposeHashWithBuffer preimage (process/message.go:60-78)."""
    assert len(value) == 32
    return be64(height) + be64(round_) + be64(valid_round) + value


def sha256(b: bytes) -> bytes:
    return hashlib.sha256(b).digest()


def message_digest(mtype: int, height: int, round_: int, valid_round: int, value: bytes) -> bytes:
    if mtype == PROPOSE:
        return sha256(propose_preimage(height, round_, valid_round, value))
    return sha256(vote_preimage(height, round_, value))


# ---------------------------------------------------------------------------
# affine point arithmetic (None = point at infinity)
Point = Optional[Tuple[int, int]]


def _inv(x: int, m: int) -> int:
    return pow(x, -1, m)


def point_add(a: Point, b: Point) -> Point:
    if a is None:
        return b
    if b is None:
        return a
    (x1, y1), (x2, y2) = a, b
    if x1 == x2:
        if (y1 + y2) % P == 0:
            return None
        lam = (3 * x1 * x1) * _inv(2 * y1, P) % P
    else:
        lam = (y2 - y1) * _inv(x2 - x1, P) % P
    x3 = (lam * lam - x1 - x2) % P
    return (x3, (lam * (x1 - x3) - y1) % P)


def point_mul(k: int, pt: Point) -> Point:
    acc: Point = None
    add = pt
    while k:
        if k & 1:
            acc = point_add(acc, add)
        add = point_add(add, add)
        k >>= 1
    return acc


G = (GX, GY)


def point_neg(a: Point) -> Point:
    return None if a is None else (a[0], (-a[1]) % P)


def lift_x(x: int, odd: int) -> Point:
    """secp256k1_ge_set_xo_var: sqrt via (p+1)/4 (p = 3 mod 4)."""
    y2 = (x * x * x + 7) % P
    y = pow(y2, (P + 1) // 4, P)
    if y * y % P != y2:
        return None
    if (y & 1) != odd:
        y = P - y
    return (x, y)


PUBKEY_UNCOMPRESSED, PUBKEY_COMPRESSED, PUBKEY_RAW64, PUBKEY_XY_STRIPPED = 0, 1, 2, 3   # include/hd_verify.h


def go_big_bytes(v: int) -> bytes:
    """Go's big.Int.Bytes(): minimal big-endian, no leading zero bytes."""
    return v.to_bytes((v.bit_length() + 7) // 8, "big")


def pubkey_bytes(q: Tuple[int, int], compressed=True) -> bytes:
    """The pubkey encoding id.NewSignatory hashes.  `compressed`: True / 1 =
    SEC1 compressed (33 B), False / 0 = SEC1 uncompressed (65 B), 2 = raw
    X || Y (64 B), 3 = X.Bytes() || Y.Bytes() (`append(pub.X.Bytes(),
    pub.Y.Bytes()...)`, leading zero bytes of each coordinate dropped)."""
    x, y = q
    if int(compressed) == PUBKEY_XY_STRIPPED:
        return go_big_bytes(x) + go_big_bytes(y)
    if int(compressed) == PUBKEY_RAW64:
        return x.to_bytes(32, "big") + y.to_bytes(32, "big")
    if compressed:
        return bytes([2 | (y & 1)]) + x.to_bytes(32, "big")
    return b"\x04" + x.to_bytes(32, "big") + y.to_bytes(32, "big")


def signatory_of_pub(q: Tuple[int, int], compressed: bool = True) -> bytes:
    """id.NewSignatory: SHA-256 of the pubkey encoding [renproject/id v0.4.2]."""
    return sha256(pubkey_bytes(q, compressed))


# ---------------------------------------------------------------------------
# recovery -- libsecp256k1 semantics as reached through go-ethereum v1.9.5
def recover(digest: bytes, sig: bytes) -> Tuple[int, Point]:
    """Return (verdict, Q).  Order of checks follows go-ethereum
    crypto/secp256k1 checkSignature (V >= 4 rejected), then libsecp256k1
    parse_compact (r, s overflow), sig_recover (zero r/s, x = r + n range,
    x on curve, Q = infinity).  High-S is accepted."""
    assert len(digest) == 32 and len(sig) == 65
    v = sig[64]
    if v >= 4:
        return BAD_RECID, None
    r = int.from_bytes(sig[0:32], "big")
    s = int.from_bytes(sig[32:64], "big")
    if r >= N or s >= N:
        return BAD_RS, None
    if r == 0 or s == 0:
        return BAD_RS, None
    x = r
    if v & 2:
        if x >= P - N:
            return NO_POINT, None
        x += N
    R = lift_x(x, v & 1)
    if R is None:
        return NO_POINT, None
    m = int.from_bytes(digest, "big") % N
    rinv = _inv(r, N)
    u1 = (-m * rinv) % N
    u2 = (s * rinv) % N
    Q = point_add(point_mul(u1, G), point_mul(u2, R))
    if Q is None:
        return INFINITY, None
    return VALID, Q


# ---------------------------------------------------------------------------
# signing (fixture construction only) -- libsecp256k1 RFC6979 + low-S
def _hmac(k: bytes, m: bytes) -> bytes:
    return hmac.new(k, m, hashlib.sha256).digest()


def rfc6979_nonce(key32: bytes, msg32: bytes, counter: int) -> bytes:
    """libsecp256k1 nonce_function_rfc6979 with no extra data / algo16."""
    v = b"\x01" * 32
    k = b"\x00" * 32
    seed = key32 + msg32
    k = _hmac(k, v + b"\x00" + seed)
    v = _hmac(k, v)
    k = _hmac(k, v + b"\x01" + seed)
    v = _hmac(k, v)
    out = b""
    for i in range(counter + 1):
        if i > 0:
            k = _hmac(k, v + b"\x00")
            v = _hmac(k, v)
        v = _hmac(k, v)
        out = v
    return out


def sign(sk: int, digest: bytes) -> bytes:
    assert 0 < sk < N
    key32 = sk.to_bytes(32, "big")
    m = int.from_bytes(digest, "big") % N
    counter = 0
    while True:
        k = int.from_bytes(rfc6979_nonce(key32, digest, counter), "big")
        counter += 1
        if k == 0 or k >= N:
            continue
        R = point_mul(k, G)
        rx = R[0]
        recid = (R[1] & 1) | (2 if rx >= N else 0)
        r = rx % N
        s = _inv(k, N) * (m + r * sk) % N
        if r == 0 or s == 0:
            continue
        if s > N // 2:
            s = N - s
            recid ^= 1
        return r.to_bytes(32, "big") + s.to_bytes(32, "big") + bytes([recid])


def pubkey_of(sk: int) -> Tuple[int, int]:
    return point_mul(sk, G)


# ---------------------------------------------------------------------------
# synthetic workload definition; mirrored bit-for-bit by
# hyperdrive_amd/csrc/hd_gen.h -- the tests compare the two.
SEED = 0x48595045


def splitmix64(x: int) -> int:
    z = (x + 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


_SEED_MIX = splitmix64(SEED)


def rnd(i: int, stream: int) -> int:
    """Counter-based stream: word ``stream`` (0..15) of message ``i``."""
    return splitmix64(_SEED_MIX ^ (((i << 4) | stream) & M64))


def signer_sk(i: int) -> int:
    """sk_i = (SHA-256("hd-sk" || BE32(i)) mod (n-1)) + 1."""
    h = int.from_bytes(sha256(b"hd-sk" + struct.pack(">I", i & 0xFFFFFFFF)), "big")
    return h % (N - 1) + 1


def canonical_value(height: int, round_: int) -> bytes:
    return sha256(b"hd-v" + be64(height) + be64(round_))


def random_value(i: int) -> bytes:
    return b"".join(struct.pack(">Q", rnd(i, 1 + j)) for j in range(4))


def vote_value(i: int, height: int, round_: int) -> bytes:
    u = rnd(i, 0) % 100
    if u < 90:
        return canonical_value(height, round_)
    if u < 95:
        return NIL_VALUE
    return random_value(i)


@dataclass
class Batch:
    """Structure-of-arrays batch (the hd_batch layout of include/hd_verify.h)."""
    mtype: List[int] = field(default_factory=list)
    height: List[int] = field(default_factory=list)
    round: List[int] = field(default_factory=list)
    valid_round: List[int] = field(default_factory=list)
    value: List[bytes] = field(default_factory=list)
    frm: List[bytes] = field(default_factory=list)
    sig: List[bytes] = field(default_factory=list)

    def __len__(self) -> int:
        return len(self.mtype)

    def append(self, mtype, height, round_, valid_round, value, frm, sig):
        self.mtype.append(mtype)
        self.height.append(height)
        self.round.append(round_)
        self.valid_round.append(valid_round)
        self.value.append(value)
        self.frm.append(frm)
        self.sig.append(sig)


# workload kinds (hd_gen_config.kind)
GEN_VOTES = 0     # C2 / C4: signer = i % S, type = 2 + (i/S)%2, h = 1 + i/(2S), r = 0
GEN_ROUNDS = 1    # C3: h = 1, per round: 1 propose + S prevotes + S precommits

NONADMITTED_BASE = 1_000_000
N_ADV_CLASSES = 13


def base_message(kind: int, i: int, S: int):
    """Uncorrupted message i: (type, h, r, vr, value, signer_index)."""
    if kind == GEN_VOTES:
        signer = i % S
        mtype = PREVOTE + ((i // S) % 2)
        h = 1 + i // (2 * S)
        r = 0
        return mtype, h, r, INVALID_ROUND, vote_value(i, h, r), signer
    per = 1 + 2 * S
    r = i // per
    k = i % per
    h = 1
    if k == 0:
        return PROPOSE, h, r, INVALID_ROUND, canonical_value(h, r), (h + r) % S
    if k <= S:
        return PREVOTE, h, r, INVALID_ROUND, vote_value(i, h, r), k - 1
    return PRECOMMIT, h, r, INVALID_ROUND, vote_value(i, h, r), k - S - 1


class KeyCache:
    def __init__(self, compressed: bool = True):
        self.compressed = compressed
        self._sk: Dict[int, int] = {}
        self._sig: Dict[int, bytes] = {}

    def sk(self, idx: int) -> int:
        if idx not in self._sk:
            self._sk[idx] = signer_sk(idx)
        return self._sk[idx]

    def signatory(self, idx: int) -> bytes:
        if idx not in self._sig:
            self._sig[idx] = signatory_of_pub(pubkey_of(self.sk(idx)), self.compressed)
        return self._sig[idx]


def _is_qr(a: int) -> bool:
    return pow(a % P, (P - 1) // 2, P) in (0, 1)


def gen_message(kind: int, i: int, S: int, adv_pct: int, keys: KeyCache):
    """Message i of the seeded workload (optionally adversarial)."""
    mtype, h, r, vr, value, signer = base_message(kind, i, S)
    cls = -1
    if adv_pct and rnd(i, 5) % 100 < adv_pct:
        cls = rnd(i, 6) % N_ADV_CLASSES
    w = rnd(i, 8)
    sk_idx = signer
    if cls in (11, 12) and i > 0:
        # double vote (11: conflicting value, 12: identical copy) of message i-1
        mtype, h, r, vr, v0, signer = base_message(kind, i - 1, S)
        sk_idx = signer
        value = v0 if cls == 12 else random_value(i)
    if cls == 6:
        sk_idx = NONADMITTED_BASE + (i % 16)
    frm = keys.signatory(sk_idx)
    sign_h = h + 1 if cls == 7 else h
    digest = message_digest(mtype, sign_h, r, vr, value)
    sig = bytearray(sign(keys.sk(sk_idx), digest))
    if cls == 0:
        raw = b"".join(struct.pack(">Q", rnd(i, 7 + j)) for j in range(9))
        sig = bytearray(raw[:65])
    elif cls == 1:
        sig[64] = 4 + (w % 252)
    elif cls == 2:
        if w & 1:
            sig[0:32] = bytes(32)
        else:
            sig[32:64] = bytes(32)
    elif cls == 3:
        bad = (N + ((w >> 1) & 0xFFFF)).to_bytes(32, "big")
        if w & 1:
            sig[0:32] = bad
        else:
            sig[32:64] = bad
    elif cls == 4:
        sig[64] |= 2
        sig[0:32] = ((P - N) + (w % (1 << 64))).to_bytes(32, "big")
    elif cls == 5:
        x = w
        while _is_qr(x * x * x + 7):
            x += 1
        sig[0:32] = x.to_bytes(32, "big")
        sig[64] &= 1
    elif cls == 8:
        if mtype in (PREVOTE, PRECOMMIT):
            mtype = PREVOTE if mtype == PRECOMMIT else PRECOMMIT
        else:
            cls = 9
    if cls == 9:
        s = int.from_bytes(sig[32:64], "big")
        sig[32:64] = (N - s).to_bytes(32, "big")
        sig[64] ^= 1
    elif cls == 10:
        k = w % (N - 1) + 1
        R = point_mul(k, G)
        m = int.from_bytes(digest, "big") % N
        s = m * _inv(k, N) % N
        if R[0] < N and s != 0:
            sig[0:32] = R[0].to_bytes(32, "big")
            sig[32:64] = s.to_bytes(32, "big")
            sig[64] = R[1] & 1
    return mtype, h, r, vr, value, frm, bytes(sig), cls


def gen_batch(kind: int, n: int, S: int, adv_pct: int = 0, start: int = 0,
              keys: Optional[KeyCache] = None) -> Tuple[Batch, List[int]]:
    keys = keys or KeyCache()
    b = Batch()
    classes = []
    for i in range(start, start + n):
        mtype, h, r, vr, value, frm, sig, cls = gen_message(kind, i, S, adv_pct, keys)
        b.append(mtype, h, r, vr, value, frm, sig)
        classes.append(cls)
    return b, classes


def admitted_set(S: int, keys: Optional[KeyCache] = None) -> List[bytes]:
    keys = keys or KeyCache()
    return [keys.signatory(j) for j in range(S)]


# ---------------------------------------------------------------------------
# verification of a batch (the VerifyBatch contract)
def verify_message(mtype, height, round_, valid_round, value, frm, sig,
                   admitted: set, compressed: bool = True) -> Tuple[int, Optional[bytes]]:
    if mtype not in (PROPOSE, PREVOTE, PRECOMMIT):
        return BAD_TYPE, None
    digest = message_digest(mtype, height, round_, valid_round, value)
    verdict, Q = recover(digest, sig)
    if verdict != VALID:
        return verdict, None
    got = signatory_of_pub(Q, compressed)
    if got != frm:                       # message_test.go:154 Equal
        return SIGNATORY_MISMATCH, got
    if frm not in admitted:              # mq/mq.go:49-51 procsAllowed
        return NOT_ADMITTED, got
    return VALID, got


def verify_batch(b: Batch, admitted: Sequence[bytes], compressed: bool = True):
    aset = set(admitted)
    verdicts, recovered = [], []
    for i in range(len(b)):
        v, got = verify_message(b.mtype[i], b.height[i], b.round[i], b.valid_round[i],
                                b.value[i], b.frm[i], b.sig[i], aset, compressed)
        verdicts.append(v)
        recovered.append(got if got is not None else bytes(32))
    return verdicts, recovered


# ---------------------------------------------------------------------------
# tally -- restates process.go insertPrevote/insertPrecommit (823-892) per
# (height, round) and the counting loops of the 2f+1 / f+1 rules.
@dataclass
class Tally:
    # (h, r, type, value) -> number of first-wins votes for value
    count: Dict[Tuple[int, int, int, bytes], int]
    # (h, r, type) -> len(PrevoteLogs[r]) / len(PrecommitLogs[r])
    distinct: Dict[Tuple[int, int, int], int]
    # (h, r) -> |TraceLogs[r]| restricted to votes (proposes are host-side)
    distinct_any: Dict[Tuple[int, int], int]
    # per message: 0 = logged, 1 = identical duplicate dropped, 2 = conflicting
    # duplicate (CatchDoublePrevote/Precommit), 3 = not a tally candidate
    dup: List[int]


def tally(b: Batch, verdicts: Sequence[int]) -> Tally:
    logs: Dict[Tuple[int, int, int], Dict[bytes, int]] = {}
    trace: Dict[Tuple[int, int], set] = {}
    dup = [3] * len(b)
    for i in range(len(b)):
        t = b.mtype[i]
        if verdicts[i] != VALID or t not in (PREVOTE, PRECOMMIT):
            continue
        key = (b.height[i], b.round[i], t)
        log = logs.setdefault(key, {})
        if b.frm[i] in log:                          # process.go:834-845
            j = log[b.frm[i]]
            dup[i] = 1 if b.value[j] == b.value[i] else 2
            continue
        log[b.frm[i]] = i                            # process.go:847
        dup[i] = 0
        trace.setdefault((b.height[i], b.round[i]), set()).add(b.frm[i])
    count: Dict[Tuple[int, int, int, bytes], int] = {}
    distinct: Dict[Tuple[int, int, int], int] = {}
    for (h, r, t), log in logs.items():
        distinct[(h, r, t)] = len(log)
        for j in log.values():                       # process.go:574-579
            k = (h, r, t, b.value[j])
            count[k] = count.get(k, 0) + 1
    return Tally(count, distinct, {k: len(v) for k, v in trace.items()}, dup)


def thresholds(n_signatories: int) -> Tuple[int, int, int]:
    """f = len(signatories)/3 (replica/replica.go:54); 2f+1 and f+1."""
    f = n_signatories // 3
    return f, 2 * f + 1, f + 1


def decide_round(t: Tally, h: int, r: int, f: int, propose_value: Optional[bytes],
                 propose_valid: bool, propose_valid_round: int = INVALID_ROUND,
                 propose_signer_new: bool = False) -> Dict[str, bool]:
    """The count predicates of the 2f+1 / f+1 rules for one (h, r), evaluated on
    the batch's final logs (the automaton's step/once-flag gating stays with the
    caller)."""
    q = 2 * f + 1
    pv = lambda v: t.count.get((h, r, PREVOTE, v), 0)
    pc = lambda v: t.count.get((h, r, PRECOMMIT, v), 0)
    out = {
        # L34 process.go:534
        "timeout_prevote": t.distinct.get((h, r, PREVOTE), 0) >= q,
        # L44 process.go:626-632
        "precommit_nil": pv(NIL_VALUE) >= q,
        # L47 process.go:658 is `len(PrecommitLogs[cur]) == 2f+1`, tried after
        # every precommit insert: over a batch's final logs it held at some
        # insert iff the final length is >= 2f+1 ("reached") ...
        "timeout_precommit_reached": t.distinct.get((h, r, PRECOMMIT), 0) >= q,
        # ... while StartRound (process.go:310) evaluates it once on entering
        # the round: only exactly 2f+1 buffered precommits fire it ("exact")
        "timeout_precommit_exact": t.distinct.get((h, r, PRECOMMIT), 0) == q,
        # L55 process.go:751 (votes plus a valid propose from a new signer)
        "skip": t.distinct_any.get((h, r), 0) + (1 if propose_signer_new else 0) >= f + 1,
        "precommit_value": False,
        "commit": False,
        "prevote_validround": False,
    }
    if propose_value is not None and propose_valid:
        out["precommit_value"] = pv(propose_value) >= q     # L36 process.go:574-582
        out["commit"] = pc(propose_value) >= q              # L49 process.go:696-702
    if propose_value is not None and propose_valid_round > INVALID_ROUND:
        out["prevote_validround"] = t.count.get((h, propose_valid_round, PREVOTE, propose_value), 0) >= q  # L28 486-494
    return out
