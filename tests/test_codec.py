"""Batch surge codec (include/hd_codec.h) against the CPU restatement
(oracle/surge_codec.py) of process/message.go Marshal / Unmarshal.

CPU: the restatement's layout (80 / 88 bytes, BE64 fields) and its relation to
the digest preimages (NewPrevoteHash hashes the first 48 bytes of a Prevote's
encoding minus From, message.go:172-186; NewProposeHash the first 56).
GPU: marshal == the restatement byte for byte; unmarshal(restatement bytes)
== the batch; round trips for all three types with and without signatures;
truncated buffers (message_test.go:65-127's "too small" cases) mark exactly
the incomplete records; bad type / unaligned pointers are argument errors."""
import numpy as np
import pytest

import surge_codec as SC


def _rand_batch(n, seed, mtype):
    rng = np.random.default_rng(seed)
    edges = np.array([0, 1, -1, 2 ** 63 - 1, -2 ** 63], dtype=np.int64)
    h = rng.integers(-2 ** 63, 2 ** 63 - 1, n, dtype=np.int64, endpoint=True)
    r = rng.integers(-2 ** 63, 2 ** 63 - 1, n, dtype=np.int64, endpoint=True)
    vr = rng.integers(-1, 100, n, dtype=np.int64)
    k = min(n, 5)
    h[:k], r[:k], vr[:k] = edges[:k], edges[::-1][:k], edges[:k]
    value = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    frm = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    sig = rng.integers(0, 256, (n, 65), dtype=np.uint8)
    typ = np.full(n, mtype, np.uint8)
    return typ, h, r, vr, value, frm, sig


def test_record_layout(oracle):
    v = bytes(range(32))
    f = bytes(range(32, 64))
    pv = SC.marshal(SC.PREVOTE, 5, -1, -1, v, f)
    assert len(pv) == 80 and pv[:8] == (5).to_bytes(8, "big") and pv[8:16] == b"\xff" * 8
    assert pv[16:48] == v and pv[48:] == f
    assert pv[:48] == oracle.vote_preimage(5, -1, v)
    pp = SC.marshal(SC.PROPOSE, 7, 2, -1, v, f, bytes(65))
    assert len(pp) == 88 + 65 and pp[:56] == oracle.propose_preimage(7, 2, -1, v)
    assert SC.unmarshal(SC.PROPOSE, pp, True) == (7, 2, -1, v, f, bytes(65))
    assert SC.unmarshal(SC.PREVOTE, pv[:79], False) is None
    assert SC.record_size(4, True) == 0 and SC.record_size(3, False) == 80


def test_abi_record_size():
    from hyperdrive_amd import _lib
    lib = _lib.load()
    for t in (1, 2, 3):
        for s in (0, 1):
            assert lib.hd_record_size(t, s) == SC.record_size(t, bool(s))
    assert lib.hd_record_size(0, 0) == 0 and lib.hd_record_size(4, 1) == 0


@pytest.fixture(scope="module")
def verifier(gpu):
    v = gpu.Verifier(0)
    yield v
    v.close()


def _device_batch(arrs):
    import torch
    from hyperdrive_amd.device import DeviceBatch
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    typ, h, r, vr, value, frm, sig = arrs
    return DeviceBatch(len(typ), t(typ), t(h), t(r), t(vr), t(value), t(frm), t(sig))


@pytest.mark.gpu
@pytest.mark.parametrize("mtype", [1, 2, 3])
@pytest.mark.parametrize("with_sig", [True, False])
@pytest.mark.parametrize("n", [1, 255, 257, 5000])
def test_marshal_unmarshal_parity(verifier, mtype, with_sig, n):
    import torch
    from hyperdrive_amd.codec import marshal_device, unmarshal_device
    arrs = _rand_batch(n, 100 * mtype + n, mtype)
    typ, h, r, vr, value, frm, sig = arrs
    want = SC.marshal_array(mtype, h, r, vr, value, frm, sig if with_sig else None)
    db = _device_batch(arrs)
    buf = marshal_device(verifier, mtype, db, with_sig)
    assert buf.cpu().numpy().tobytes() == want
    wire = torch.from_numpy(np.frombuffer(want, np.uint8).copy()).cuda()
    out, status = unmarshal_device(verifier, mtype, wire, n, with_sig)
    assert int(status.sum()) == 0
    hb = out.to_host()
    assert (hb.type == mtype).all()
    assert hb.height.tolist() == h.tolist() and hb.round.tolist() == r.tolist()
    if mtype == 1:
        assert hb.valid_round.tolist() == vr.tolist()
    else:
        assert (hb.valid_round == -1).all()
    assert hb.value.tobytes() == value.tobytes() and hb.frm.tobytes() == frm.tobytes()
    if with_sig:
        assert hb.sig.tobytes() == sig.tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("cut", [1, 79, 80, 81, 145 * 3 + 17])
def test_truncated_buffer(verifier, cut):
    import torch
    from hyperdrive_amd.codec import unmarshal_device
    n = 600
    arrs = _rand_batch(n, 9, 2)
    typ, h, r, vr, value, frm, sig = arrs
    full = SC.marshal_array(2, h, r, None, value, frm, sig)
    short = full[: len(full) - cut]
    wire = torch.zeros(len(full) + 16, dtype=torch.uint8).cuda()
    wire[: len(short)] = torch.from_numpy(np.frombuffer(short, np.uint8).copy()).cuda()
    out, status = unmarshal_device(verifier, 2, wire[: len(short)], n, True)
    want = [0 if rec is not None else 1 for rec in SC.unmarshal_array(2, short, n, True)]
    assert status.cpu().numpy().tolist() == want
    hb = out.to_host()
    ok = np.array(want) == 0
    assert hb.height[ok].tolist() == h[ok].tolist()
    assert (hb.height[~ok] == 0).all() and (hb.sig[~ok] == 0).all()


@pytest.mark.gpu
def test_argument_errors(verifier):
    import ctypes
    import torch
    from hyperdrive_amd import _lib
    from hyperdrive_amd.codec import unmarshal_device
    lib = _lib.load()
    buf = torch.zeros(1024, dtype=torch.uint8).cuda()
    with pytest.raises(_lib.HDError):
        unmarshal_device(verifier, 4, buf, 3)
    with pytest.raises(_lib.HDError):
        unmarshal_device(verifier, 2, buf[1:], 3)     # unaligned
    assert lib.hd_unmarshal_batch_device(verifier.handle, 2, 1, None, 0, 0, ctypes.byref(_lib.HdBatchOut()), None,
                                         None) == 0   # n == 0 is a no-op
