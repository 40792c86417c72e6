"""Known-key fast path (hd_fixedbase.h, hd_fastverify.hip).

The fast path may only answer VALID when the full recovery would return
exactly the known key, and otherwise must either give the reference's early
verdict (BAD_RECID, BAD_RS, NO_POINT for r + n >= p) or hand the message to
the full recovery.  CPU: the device header built for the host, against the
oracle's recovery (oracle/hd_pyoracle.py), on honest, malleated, wrong-key,
wrong-digest, wrong-parity, malformed and r + n signatures, and the table
layout against oracle point multiplication.  GPU: verifying a batch with the
fast path (keys learned on the first pass) gives bit-identical verdicts,
recovered signatories, signer indices and bitmaps to the full recovery
alone (HD_VERIFY_FASTPATH=0) on the adversarial mix, and the second pass
really takes the fast path."""
import ctypes
import os
import random

import numpy as np
import pytest

NEEDS_SLOW = 0xFE


@pytest.fixture(scope="module")
def fb(hostmath):
    L = hostmath.L
    L.hdh_fb_verify.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p]
    L.hdh_fb_verify.restype = ctypes.c_int
    L.hdh_fb_entry.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_uint32, ctypes.c_char_p]
    return L


def _pub64(q):
    return q[0].to_bytes(32, "big") + q[1].to_bytes(32, "big")


def _verify(fb, q, digest, sig):
    return fb.hdh_fb_verify(_pub64(q), digest, sig)


def test_table_entries_are_window_multiples(fb, oracle):
    O = oracle
    for j, d in [(0, 1), (0, 2048), (1, 1), (7, 1234), (21, 1), (21, 16)]:
        out = ctypes.create_string_buffer(64)
        fb.hdh_fb_entry(_pub64((O.GX, O.GY)), j, d, out)
        want = O.point_mul(d << (12 * j), (O.GX, O.GY))
        assert out.raw == _pub64(want), (j, d)


def test_scalar_montgomery(fb, oracle):
    """sm_mul (hd_scmont.h, k_fast_scalars' products): a b 2^-261 mod n for
    random and extreme operands, and chains whose intermediate values stay in
    [0, 2n) -- against Python integers."""
    O = oracle
    n = O.N
    Rinv = pow(1 << 261, -1, n)
    fb.hdh_sm_mul.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_void_p]
    fb.hdh_sm_chain.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p]
    rng = random.Random(9)
    vals = [0, 1, 2, n - 1, n - 2, (1 << 255), n >> 1] + [rng.randrange(n) for _ in range(60)]
    out = ctypes.create_string_buffer(32)
    for k in range(len(vals) - 1):
        a, b = vals[k], vals[k + 1]
        fb.hdh_sm_mul(a.to_bytes(32, "big"), b.to_bytes(32, "big"), out, None)
        assert int.from_bytes(out.raw, "big") == a * b * Rinv % n, (a, b)
    for t in range(20):
        x = rng.randrange(1, n)
        ys = [rng.randrange(1, n) if t % 3 else n - 1 for _ in range(12)]
        fb.hdh_sm_chain(x.to_bytes(32, "big"), b"".join(y.to_bytes(32, "big") for y in ys), len(ys), out)
        want = x
        for y in ys:
            want = want * y * Rinv % n
        assert int.from_bytes(out.raw, "big") == want


def test_first_step_addition(fb, oracle):
    """gej_add_ge_z1 (the fixed-base sum's first addition, two affine points)
    against oracle point addition; a = +-b yields Z3 = 0 (the check then hands
    the message to the full recovery)."""
    O = oracle
    fb.hdh_add_affine.argtypes = [ctypes.c_char_p] * 4 + [ctypes.c_char_p]
    fb.hdh_add_affine.restype = ctypes.c_int
    rng = random.Random(5)
    b32 = lambda v: v.to_bytes(32, "big")
    for _ in range(40):
        a = O.point_mul(rng.randrange(1, O.N), (O.GX, O.GY))
        b = O.point_mul(rng.randrange(1, O.N), (O.GX, O.GY))
        out = ctypes.create_string_buffer(64)
        assert fb.hdh_add_affine(b32(a[0]), b32(a[1]), b32(b[0]), b32(b[1]), out) == 0
        assert out.raw == _pub64(O.point_add(a, b))
    a = O.point_mul(7, (O.GX, O.GY))
    na = O.point_neg(a)
    out = ctypes.create_string_buffer(64)
    assert fb.hdh_add_affine(b32(a[0]), b32(a[1]), b32(na[0]), b32(na[1]), out) == 1
    assert fb.hdh_add_affine(b32(a[0]), b32(a[1]), b32(a[0]), b32(a[1]), out) == 1


def _xyzz_sum(fb, pts, neg, skip, force_rare=0):
    fb.hdh_xyzz_sum.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p,
                                ctypes.c_int]
    fb.hdh_xyzz_sum.restype = ctypes.c_int
    n = len(pts)
    out = ctypes.create_string_buffer(64)
    ng = np.asarray(neg, np.int32)
    sk = np.asarray(skip, np.int32)
    deg = fb.hdh_xyzz_sum(b"".join(_pub64(p) for p in pts), ng.ctypes.data, sk.ctypes.data, n, out, force_rare)
    return None if deg else (int.from_bytes(out.raw[:32], "big"), int.from_bytes(out.raw[32:], "big"))


def test_xyzz_sums(fb, oracle):
    """k_fast_sums' XYZZ accumulation (gxz_add_ge_z1, gxz_add_ge_nx, the
    zero-digit selects, gxz_finish) on the host against oracle point
    addition: 24 points (the 11 + 13 windows of C2) with random signs and
    rare skips, skipped first windows, and the degenerate sums (a partial sum
    equal to +-the next point) that must end with ZZ = 0."""
    O = oracle
    rng = random.Random(77)
    G = (O.GX, O.GY)
    for t in range(30):
        n = 24
        pts = [O.point_mul(rng.randrange(1, O.N), G) for _ in range(n)]
        neg = [rng.random() < 0.5 for _ in range(n)]
        skip = [rng.random() < (0.3 if t % 5 == 0 else 0.02) for _ in range(n)]
        if t % 7 == 0:
            skip[0] = True
        if t % 11 == 0:
            skip[0] = skip[1] = True
        want = None
        for p, ng, sk in zip(pts, neg, skip):
            if sk:
                continue
            q = O.point_neg(p) if ng else p
            want = q if want is None else O.point_add(want, q)
        for force in (0, 1):   # the repair branch where this lane needs it / at every step
            got = _xyzz_sum(fb, pts, [int(x) for x in neg], [int(x) for x in skip], force)
            if want is None:
                assert got is None
            else:
                assert got == want, (t, force)
    # degenerate: the partial sum equals +-the next point (doubling / cancel)
    a = O.point_mul(12345, G)
    b = O.point_mul(777, G)
    ab = O.point_add(a, b)
    for nxt, ng in [(ab, 0), (ab, 1)]:
        assert _xyzz_sum(fb, [a, b, nxt, O.point_mul(5, G)], [0, 0, ng, 0], [0, 0, 0, 0]) is None
    # the affine first addition's own degenerate cases
    assert _xyzz_sum(fb, [a, a], [0, 1], [0, 0]) is None
    assert _xyzz_sum(fb, [a, a, b], [0, 0, 0], [0, 0, 0]) is None
    # a skipped second window, then the general addition from an affine start
    for force in (0, 1):
        assert _xyzz_sum(fb, [a, b, b], [0, 0, 1], [0, 1, 0], force) == O.point_add(a, O.point_neg(b))
    # a skipped window's point is never added: a sum equal to +-that point
    # stays exact
    for force in (0, 1):
        assert _xyzz_sum(fb, [a, b, ab, b], [0, 0, 0, 0], [0, 0, 1, 0], force) == O.point_add(ab, b)


def test_fast_path_agrees_with_recovery(fb, oracle):
    O = oracle
    rng = random.Random(12)
    sk = O.signer_sk(3)
    P = O.pubkey_of(sk)
    other = O.pubkey_of(O.signer_sk(4))
    n_valid = 0
    for t in range(60):
        digest = bytes(rng.randrange(256) for _ in range(32))
        sig = O.sign(sk, digest)
        kind = t % 6
        if kind == 1:                       # high-S malleation: still recovers P
            s = O.N - int.from_bytes(sig[32:64], "big")
            sig = sig[:32] + s.to_bytes(32, "big") + bytes([sig[64] ^ 1])
        elif kind == 2:                     # wrong parity: another key
            sig = sig[:64] + bytes([sig[64] ^ 1])
        elif kind == 3:                     # another digest
            digest = bytes(rng.randrange(256) for _ in range(32))
        elif kind == 4:                     # another signer's key
            sig = O.sign(O.signer_sk(4), digest)
        elif kind == 5:                     # random r, s
            sig = rng.randrange(1, O.N).to_bytes(32, "big") + rng.randrange(1, O.N).to_bytes(32, "big") + \
                bytes([rng.randrange(2)])
        v, q = O.recover(digest, sig)
        got = _verify(fb, P, digest, sig)
        if v == O.VALID and q == P:
            assert got == O.VALID, t
            n_valid += 1
        else:
            assert got == NEEDS_SLOW, (t, v)
        if kind == 4:
            assert _verify(fb, other, digest, sig) == O.VALID
    assert n_valid >= 20


def test_early_verdicts_match_recovery(fb, oracle):
    O = oracle
    P = O.pubkey_of(O.signer_sk(3))
    d = bytes(range(32))
    good = O.sign(O.signer_sk(3), d)
    r, s = good[:32], good[32:64]
    cases = [
        (r + s + bytes([4]), O.BAD_RECID),
        (r + s + bytes([255]), O.BAD_RECID),
        (bytes(32) + s + bytes([0]), O.BAD_RS),
        (r + bytes(32) + bytes([1]), O.BAD_RS),
        (O.N.to_bytes(32, "big") + s + bytes([0]), O.BAD_RS),
        (r + O.N.to_bytes(32, "big") + bytes([0]), O.BAD_RS),
        ((O.P - O.N).to_bytes(32, "big") + s + bytes([2]), O.NO_POINT),
        ((O.N - 1).to_bytes(32, "big") + s + bytes([3]), O.NO_POINT),
    ]
    for sig, want in cases:
        assert O.recover(d, sig)[0] == want
        assert _verify(fb, P, d, sig) == want


def test_r_plus_n_recovery_to_the_known_key(fb, oracle):
    """v & 2 (x = r + n): craft R with x >= n, any s; the key it recovers to
    is then the known key, and the fast path must accept exactly it."""
    O = oracle
    rng = random.Random(5)
    for _ in range(200):
        r = rng.randrange(1, O.P - O.N)
        R = O.lift_x(r + O.N, 0)
        if R is not None:
            break
    digest = bytes(rng.randrange(256) for _ in range(32))
    s = rng.randrange(1, O.N)
    sig = r.to_bytes(32, "big") + s.to_bytes(32, "big") + bytes([2])
    v, q = O.recover(digest, sig)
    assert v == O.VALID
    assert _verify(fb, q, digest, sig) == O.VALID
    assert _verify(fb, q, digest, sig[:64] + bytes([3])) == NEEDS_SLOW


# ---------------------------------------------------------------- GPU
def _run(v, db, n):
    import torch
    from hyperdrive_amd.device import work_stream
    ws = work_stream()
    outs = [torch.empty(n, dtype=torch.uint8, device="cuda"), torch.empty(n, dtype=torch.int32, device="cuda"),
            torch.empty((n, 32), dtype=torch.uint8, device="cuda"),
            torch.zeros((n + 31) // 32, dtype=torch.int32, device="cuda")]
    v.verify_batch_device(db.c_struct(), outs[0].data_ptr(), outs[2].data_ptr(), outs[1].data_ptr(),
                          outs[3].data_ptr(), ws.cuda_stream)
    ws.synchronize()
    return outs


@pytest.mark.gpu
@pytest.mark.parametrize("compressed", [True, False, 2, 3])
@pytest.mark.parametrize("kind,S,n,adv", [(0, 100, 100_003, 30), (1, 1000, 40_000, 30), (0, 7, 5000, 0)])
def test_fast_path_equals_full_recovery(gpu, kind, S, n, adv, compressed):
    import torch
    from hyperdrive_amd.device import generate
    from hyperdrive_amd.verify import Verifier
    fast = Verifier(0, compressed=compressed)
    slow = Verifier(0, compressed=compressed)
    slow.set_fastpath(False)
    ks = fast.gen_keys(S)
    db, _, _ = generate(fast, kind, n, S, adv, keys=ks, start=4242)
    for v in (fast, slow):
        v.set_signatories(ks[0])
    ref = _run(slow, db, n)
    assert fast.known_keys() == 0
    first = _run(fast, db, n)                    # learns the keys of the signers it sees
    learned = fast.known_keys()
    fallback_first = fast.fastpath_stats()[1]
    second = _run(fast, db, n)                   # fast path for every learned signer
    fallback_second = fast.fastpath_stats()[1]
    for a, b, c in zip(ref, first, second):
        assert torch.equal(a, b) and torch.equal(a, c)
    signers_valid = len(set(ref[1][ref[0] == 0].cpu().tolist()))
    assert learned == signers_valid and slow.known_keys() == 0
    # second pass: only the non-VALID messages (minus early verdicts) fall back
    n_invalid = int((ref[0] != 0).sum())
    assert fallback_first >= n - int((ref[0] == 7).sum()) and fallback_second <= n_invalid
    assert int((ref[0] == 0).sum()) > 0
    fast.close()
    slow.close()


def test_window_digits_recode_the_scalar(fb, oracle):
    """fb_digit: signed Booth digits d_j in [-2^(W-1), 2^(W-1)], the top one
    unsigned, with sum d_j 2^(W j) == k, for random and edge scalars (host
    build, W = 12)."""
    fb.hdh_fb_digits.argtypes = [ctypes.c_char_p, ctypes.c_void_p]
    fb.hdh_fb_digits.restype = ctypes.c_int
    rng = random.Random(8)
    ks = [0, 1, oracle.N - 1, (1 << 255), (1 << 256) - 1, 0x7FF, 0x800, 0xFFF] + \
         [rng.randrange(1 << 256) for _ in range(200)]
    for k in ks:
        out = np.zeros(64, np.int32)
        nwin = fb.hdh_fb_digits(k.to_bytes(32, "big"), out.ctypes.data)
        w = 12
        assert nwin == (256 + w - 1) // w
        assert all(-(1 << (w - 1)) <= int(d) <= (1 << (w - 1)) for d in out[:nwin - 1])
        assert 0 <= int(out[nwin - 1]) <= (1 << (256 - w * (nwin - 1)))     # top window: unsigned
        assert sum(int(d) << (w * j) for j, d in enumerate(out[:nwin])) == k


def test_pairwise_check_equals_single(fb, oracle):
    """verify_fast2 (two messages per lane, one inversion of each kind for
    the pair) gives each message the verdict verify_fast gives it alone,
    whatever its partner is (ready or not, early verdict, fallback)."""
    O = oracle
    fb.hdh_fb_verify2.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_void_p, ctypes.c_char_p]
    rng = random.Random(21)
    sk = O.signer_sk(3)
    P = O.pubkey_of(sk)
    msgs = []
    for t in range(24):
        d = bytes(rng.randrange(256) for _ in range(32))
        sig = O.sign(sk, d)
        if t % 4 == 1:
            sig = sig[:64] + bytes([sig[64] ^ 1])            # fallback
        elif t % 4 == 2:
            sig = sig[:64] + bytes([7])                      # BAD_RECID
        msgs.append((d, sig))
    for a in range(0, len(msgs), 2):
        for ready in ([1, 1], [1, 0], [0, 1]):
            (da, sa), (db, sb) = msgs[a], msgs[(a + 3) % len(msgs)]
            out = ctypes.create_string_buffer(2)
            fb.hdh_fb_verify2(_pub64(P), da + db, sa + sb, np.array(ready, np.int32).ctypes.data, out)
            for k, (d, s) in enumerate([(da, sa), (db, sb)]):
                want = _verify(fb, P, d, s) if ready[k] else NEEDS_SLOW
                assert out.raw[k] == want, (a, ready, k)


@pytest.mark.gpu
@pytest.mark.parametrize("width", [13, 16, 20, 22])
def test_key_table_widths_equal_full_recovery(gpu, monkeypatch, width):
    """Every per-key table width (HD_FB_PW at context creation, then the
    key_width variant: 13-bit windows, 20 additions for u2; 16-bit, 16;
    20-bit, 13; 22-bit, 12) gives the full recovery's outputs on the adversarial mix, a
    ragged batch (n not a multiple of the 8 messages per lane of the split
    check), and after the admitted set is re-mapped at the other width (every
    key is learned again)."""
    import torch
    from hyperdrive_amd.device import generate
    from hyperdrive_amd.verify import Verifier
    monkeypatch.setenv("HD_FB_PW", str(width))
    S, n = 40, 20_011
    fast = Verifier(0)
    slow = Verifier(0)
    slow.set_fastpath(False)
    ks = fast.gen_keys(S)
    db, _, _ = generate(fast, 0, n, S, 30, keys=ks, start=777)
    for v in (fast, slow):
        v.set_signatories(ks[0])
    ref = _run(slow, db, n)
    for _ in range(2):
        got = _run(fast, db, n)
        assert all(torch.equal(a, b) for a, b in zip(ref, got))
    assert fast.known_keys() > 0 and fast.fastpath_stats()[1] <= int((ref[0] != 0).sum())
    assert fast.variant("key_width") == width
    fast.set_variant("key_width", {13: 20, 16: 13, 20: 22, 22: 16}[width])   # (the environment is read at creation only)
    fast.set_signatories(ks[0])
    assert fast.known_keys() == 0
    for _ in range(2):
        got = _run(fast, db, n)
        assert all(torch.equal(a, b) for a, b in zip(ref, got))
    assert fast.known_keys() > 0
    fast.close()
    slow.close()


@pytest.mark.gpu
@pytest.mark.parametrize("off", [1, 4, 8])
def test_misaligned_records_equal_aligned(gpu, off):
    """The record loads (hd_common.h) take 16-byte / dword vector paths only
    for aligned bases: signatures, values, Froms and the recovered-signatory
    output at byte offsets 1, 4 and 8 must give what aligned buffers give, on
    the known-key check and the full recovery alike."""
    import torch
    from hyperdrive_amd._lib import HdBatch
    from hyperdrive_amd.device import generate, work_stream
    from hyperdrive_amd.verify import Verifier
    n, S = 5003, 100
    v = Verifier(0)
    ks = v.gen_keys(S)
    v.set_signatories(ks[0])
    db, _, _ = generate(v, 0, n, S, 30, keys=ks, start=77)
    first = _run(v, db, n)                       # full recovery, learns the keys
    ref = _run(v, db, n)                         # known-key check
    for a, b in zip(first, ref):
        assert torch.equal(a, b)

    def shifted(t):
        flat = torch.zeros(t.numel() + off, dtype=torch.uint8, device="cuda")
        view = flat[off:off + t.numel()]
        view.copy_(t.reshape(-1))
        return flat, view
    keep = [shifted(db.value), shifted(db.frm), shifted(db.sig)]
    mb = HdBatch(n, db.type.data_ptr(), db.height.data_ptr(), db.round.data_ptr(), db.valid_round.data_ptr(),
                 keep[0][1].data_ptr(), keep[1][1].data_ptr(), keep[2][1].data_ptr())
    rec_flat = torch.zeros(32 * n + off, dtype=torch.uint8, device="cuda")
    verdict = torch.empty(n, dtype=torch.uint8, device="cuda")
    signer = torch.empty(n, dtype=torch.int32, device="cuda")
    bitmap = torch.zeros((n + 31) // 32, dtype=torch.int32, device="cuda")
    ws = work_stream()
    v.verify_batch_device(mb, verdict.data_ptr(), rec_flat[off:].data_ptr(), signer.data_ptr(), bitmap.data_ptr(),
                          ws.cuda_stream)
    ws.synchronize()
    assert torch.equal(verdict, ref[0]) and torch.equal(signer, ref[1]) and torch.equal(bitmap, ref[3])
    assert torch.equal(rec_flat[off:off + 32 * n].view(n, 32), ref[2])
    assert int((ref[0] == 0).sum()) > 0 and v.fastpath_stats()[1] <= int((ref[0] != 0).sum())
    v.close()


def test_infinity_from_the_g_table(fb, oracle):
    """fb_is_infinity (k_slow_lift's early INFINITY verdict for leftovers of
    the known-key check): true exactly when R == (m / s) G, i.e. when the
    reference's recovery returns the point at infinity (s R = m G); false for
    -R, for other R, and for m = 0; and the oracle's recovery agrees."""
    O = oracle
    fb.hdh_fb_is_infinity.argtypes = [ctypes.c_char_p] * 4
    fb.hdh_fb_is_infinity.restype = ctypes.c_int
    b32 = lambda v: v.to_bytes(32, "big")
    rng = random.Random(31)
    G = (O.GX, O.GY)
    for t in range(12):
        k = rng.randrange(1, O.N)
        R = O.point_mul(k, G)
        m = rng.randrange(1, O.N) if t else 0
        s = m * pow(k, -1, O.N) % O.N if m else rng.randrange(1, O.N)
        want = m != 0   # s R = m G by construction (m = 0: s R = 0 G impossible)
        assert fb.hdh_fb_is_infinity(b32(R[0]), b32(R[1]), b32(m), b32(s)) == int(want), t
        nR = O.point_neg(R)
        assert fb.hdh_fb_is_infinity(b32(nR[0]), b32(nR[1]), b32(m), b32(s)) == 0
        other = rng.randrange(1, O.N)
        assert fb.hdh_fb_is_infinity(b32(R[0]), b32(R[1]), b32(m), b32(other)) == int(other == s)
        if m and R[0] < O.N:        # the reference's recovery of (m, r = x_R, s, v = parity): infinity
            v, _ = O.recover(b32(m), b32(R[0]) + b32(s) + bytes([R[1] & 1]))
            assert v == O.INFINITY


@pytest.mark.parametrize("n", [0, 1, 2, 7, 100, 1000, 4096])
def test_admitted_index_equals_binary_search(fb, n):
    """The hashed admitted index (hd_verify_msg.h adm_index_find, used by
    k_fast_prep and the tally / route passes) returns what the binary search
    over the sorted table returns, for every member, for non-members, and for
    non-members sharing a member's first four words (the hashed prefix)."""
    fb.hdh_adm_lookup.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32,
                                  ctypes.c_void_p]
    rng = np.random.default_rng(n + 5)
    # rows sorted lexicographically (uint8: byte order), duplicates dropped
    table = np.unique(rng.integers(0, 256, (n, 32), dtype=np.uint8), axis=0)
    queries = [table.copy()] if n else []
    queries.append(rng.integers(0, 256, (257, 32), dtype=np.uint8))
    if n:
        near = table.copy()
        near[:, 31] ^= 1                  # same hashed prefix, different tail
        queries.append(near)
    q = np.ascontiguousarray(np.concatenate(queries))
    out = np.zeros(2 * len(q), np.int32)
    t = np.ascontiguousarray(table)
    fb.hdh_adm_lookup(t.ctypes.data, len(t), q.ctypes.data, len(q), out.ctypes.data)
    assert out[:len(q)].tolist() == out[len(q):].tolist()
    if n:
        assert out[:len(t)].tolist() == list(range(len(t)))


@pytest.mark.gpu
def test_budget_picks_narrow_tables_for_many_keys(gpu, monkeypatch):
    """The default width follows the table budget: with a budget that holds
    every admitted key's 13-bit tables (5 MB) but not their 16-bit ones
    (36 MB), the context takes 13-bit windows (20 key windows) and every key
    still gets a slot -- no signatory is left to the full recovery -- with the
    full recovery's outputs."""
    import torch
    from hyperdrive_amd.device import generate
    from hyperdrive_amd.verify import Verifier
    monkeypatch.setenv("HD_FB_MAX_BYTES", str(2e9))
    S, n = 100, 40_000
    fast = Verifier(0)
    slow = Verifier(0)
    slow.set_fastpath(False)
    try:
        ks = fast.gen_keys(S)
        db, _, _ = generate(fast, 0, n, S, 10, keys=ks, start=31337)
        for v in (fast, slow):
            v.set_signatories(ks[0])
        assert fast.fastpath_geometry()[1] == 20
        ref = _run(slow, db, n)
        for _ in range(3):
            got = _run(fast, db, n)
            assert all(torch.equal(a, b) for a, b in zip(ref, got))
        assert fast.known_keys() == S
        assert fast.fastpath_stats()[1] <= int((ref[0] != 0).sum()) + 5
    finally:
        fast.close()
        slow.close()


@pytest.mark.gpu
def test_failed_table_allocation_retries_narrower(gpu, monkeypatch):
    """A per-key table allocation the device refuses (HD_FB_FAIL_WIDTH: the
    library's test hook fails every table allocation at that width, as when
    another process took the memory after the width was picked): the set
    change retries at the next narrower width (20 -> 16 bits) and the
    outputs equal the full recovery's.  With the width forced
    (HD_VAR_KEY_WIDTH) there is no retry: hd_set_signatories fails with
    HD_ENOMEM, and until a set change succeeds every message takes the full
    recovery against the new set, with the same outputs; once the memory is
    there the next set change maps the tables."""
    import torch
    from hyperdrive_amd import _lib
    from hyperdrive_amd.device import generate
    from hyperdrive_amd.verify import Verifier
    monkeypatch.setenv("HD_FB_FAIL_WIDTH", "20")
    S, n = 100, 40_000
    fast, forced, slow = Verifier(0), Verifier(0), Verifier(0)
    slow.set_fastpath(False)
    forced.set_variant("key_width", 20)
    try:
        ks = fast.gen_keys(S)
        db, _, _ = generate(fast, 0, n, S, 10, keys=ks, start=4242)
        fast.set_signatories(ks[0])
        slow.set_signatories(ks[0])
        assert fast.fastpath_geometry()[1] == 16
        with pytest.raises(_lib.HDError):
            forced.set_signatories(ks[0])
        ref = _run(slow, db, n)
        for v in (fast, forced):
            for _ in range(2):
                got = _run(v, db, n)
                assert all(torch.equal(a, b) for a, b in zip(ref, got))
        assert fast.known_keys() == S
        monkeypatch.delenv("HD_FB_FAIL_WIDTH")
        forced.set_signatories(ks[0])
        assert forced.fastpath_geometry()[1] == 13
        for _ in range(3):
            got = _run(forced, db, n)
            assert all(torch.equal(a, b) for a, b in zip(ref, got))
        assert forced.known_keys() == S
    finally:
        fast.close()
        forced.close()
        slow.close()


def test_foreign_dictionary_rebuild_keeps_slot_holders(hostmath):
    """fb_evict's dictionary rebuild (hd_fixedbase.h fdict_rebuild, host
    build): Froms whose buckets collide fill one probe run of 8.  Slotless
    entries past it are dropped; a slot holder past it makes the rebuild fail,
    so the caller keeps the old dictionary instead of stranding the slot
    (ADVICE r5).  Every entry that got a bucket is found again by
    fdict_find with its slot."""
    import ctypes
    L = hostmath.L
    L.hdh_fdict_bucket.restype = ctypes.c_uint32
    L.hdh_fdict_rebuild.restype = ctypes.c_int
    L.hdh_fdict_find.restype = ctypes.c_int32
    rng = np.random.default_rng(77)
    NONE = 0xFFFFFFFF

    def bucket(f):
        return L.hdh_fdict_bucket(f.ctypes.data_as(ctypes.c_void_p))

    same = []                                   # 10 Froms in bucket 5
    while len(same) < 10:
        f = rng.integers(0, 2 ** 32, 8, dtype=np.uint64).astype(np.uint32)
        if bucket(f) == 5:
            same.append(f)
    other = [f for f in (rng.integers(0, 2 ** 32, (40, 8), dtype=np.uint64).astype(np.uint32)) if bucket(f) not in
             range(5, 13)][:5]

    def rebuild(froms, slots):
        fr = np.ascontiguousarray(np.array(froms, np.uint32).reshape(-1, 8))
        sl = np.array(slots, np.uint32)
        nd = np.zeros(10 * 128, np.uint32)
        where = np.zeros(len(slots), np.int32)
        ok = L.hdh_fdict_rebuild(fr.ctypes.data_as(ctypes.c_void_p), sl.ctypes.data_as(ctypes.c_void_p),
                                 len(slots), nd.ctypes.data_as(ctypes.c_void_p),
                                 where.ctypes.data_as(ctypes.c_void_p))
        return ok, nd, where

    def find(nd, f):
        return L.hdh_fdict_find(nd.ctypes.data_as(ctypes.c_void_p), np.ascontiguousarray(f).ctypes.data_as(
            ctypes.c_void_p))

    # 8 holders fill the run; 2 slotless colliding Froms and the others follow
    froms = same[:8] + same[8:] + other
    slots = list(range(100, 108)) + [NONE, NONE] + [NONE] * len(other)
    ok, nd, where = rebuild(froms, slots)
    assert ok == 1
    assert sorted(where[:8].tolist()) == list(range(5, 13)) and where[8:10].tolist() == [-1, -1]
    for f, s in zip(froms[:8], slots[:8]):
        assert find(nd, f) == s
    assert all(w >= 0 for w in where[10:])
    # a ninth slot holder in the same run: the rebuild refuses
    ok, _, _ = rebuild(same[:9], list(range(100, 109)))
    assert ok == 0
    # holders first: the same nine with the ninth slotless rebuild, the ninth dropped
    ok, nd, where = rebuild(same[:9], list(range(100, 108)) + [NONE])
    assert ok == 1 and where[8] == -1 and find(nd, same[8]) == -1
