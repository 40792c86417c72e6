"""Digest lanes (include/hd_digest.h, hd_keccak.h).

The reference never calls Keccak, so this lane is pinned by
public known answers and by FIPS 202 itself, not by the reference:
- the FIPS 202 restatement (oracle/keccak_oracle.py) reproduces the public
  Keccak-256 answers and hashlib.sha3_256 (same permutation, pad 0x06);
- the header the kernels run (hd_keccak.h, host build) equals the
  restatement for every length around the 136-byte rate boundary and for
  the fixed 48/56-byte preimages;
- GPU: digest lanes (SHA-256 / Keccak-256 / SHA3-256) of random batches and
  of unaligned variable-length strings equal hashlib / the restatement;
  verification over caller-supplied digests equals hd_verify_batch_device
  on SHA-256 digests and accepts signatures made over Keccak-256 digests."""
import ctypes
import hashlib
import os
import random
import struct

import numpy as np
import pytest

import keccak_oracle as K

KATS = {
    b"": "c5d2460186f7233c927e7db2dcc703c0e500b653ca82273b7bfad8045d85a470",
    b"abc": "4e03657aea45a94fc7d47ba826c8d667c0d1e6e33a64a036ec44f58fa12d6c45",
    b"The quick brown fox jumps over the lazy dog":
        "4d741b6f1eb29cb2a9b9911c82f56fa8d73b04959d3d9d222895df6c0b28aa15",
}
LENGTHS = [0, 1, 7, 8, 47, 48, 55, 56, 63, 64, 127, 134, 135, 136, 137, 200, 271, 272, 273, 500, 1000]


def test_keccak256_known_answers():
    for msg, hexd in KATS.items():
        assert K.keccak256(msg).hex() == hexd


def test_fips202_constants_and_sha3_agree_with_hashlib():
    assert K.ROUND_CONSTANTS[0] == 1 and K.ROUND_CONSTANTS[23] == 0x8000000080008008
    rng = random.Random(1)
    for n in LENGTHS:
        d = bytes(rng.randrange(256) for _ in range(n))
        assert K.sha3_256(d) == hashlib.sha3_256(d).digest(), n


@pytest.fixture(scope="module")
def hk(hostmath):
    L = hostmath.L
    L.hdh_keccak_bytes.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p]
    L.hdh_keccak_msg.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                 ctypes.c_char_p, ctypes.c_char_p]
    return L


def test_header_sponge_matches_restatement(hk):
    rng = random.Random(2)
    for pad in (0x01, 0x06):
        for n in LENGTHS:
            d = bytes(rng.randrange(256) for _ in range(n))
            out = ctypes.create_string_buffer(32)
            hk.hdh_keccak_bytes(pad, d, n, out)
            assert out.raw == K.sponge256(d, pad), (pad, n)


def test_header_preimage_lanes_match_restatement(hk):
    rng = random.Random(3)
    for _ in range(200):
        t = rng.choice([1, 2, 3])
        h, r, vr = (rng.randrange(-(1 << 63), 1 << 63) for _ in range(3))
        val = bytes(rng.randrange(256) for _ in range(32))
        for pad in (0x01, 0x06):
            out = ctypes.create_string_buffer(32)
            hk.hdh_keccak_msg(pad, t, h, r, vr, val, out)
            assert out.raw == K.sponge256(K.preimage(t, h, r, vr, val), pad)


# ---------------------------------------------------------------- GPU
@pytest.fixture(scope="module")
def verifier(gpu):
    v = gpu.Verifier(0)
    yield v
    v.close()


def _rand_batch(rng, n):
    from hyperdrive_amd.verify import Batch
    typ = rng.integers(0, 6, n).astype(np.uint8)                 # 0, 4, 5: not a message type
    ext = rng.integers(-(1 << 63), (1 << 63) - 1, (n, 3), dtype=np.int64)
    small = rng.integers(-2, 100, (n, 3))
    hrv = np.where(rng.random((n, 3)) < 0.5, ext, small).astype(np.int64)
    val = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    return Batch(typ, hrv[:, 0], hrv[:, 1], hrv[:, 2], val, np.zeros((n, 32), np.uint8), np.zeros((n, 65), np.uint8))


@pytest.mark.gpu
@pytest.mark.parametrize("algo", [0, 1, 2])
def test_gpu_preimage_digests(verifier, algo):
    from hyperdrive_amd.device import DeviceBatch
    from hyperdrive_amd.digest import digest_device
    rng = np.random.default_rng(10 + algo)
    b = _rand_batch(rng, 3001)
    d = digest_device(verifier, algo, DeviceBatch.from_host(b)).cpu().numpy()
    for i in range(len(b)):
        t = int(b.type[i])
        if t not in (1, 2, 3):
            assert not d[i].any()
            continue
        pre = K.preimage(t, int(b.height[i]), int(b.round[i]), int(b.valid_round[i]), b.value[i].tobytes())
        want = hashlib.sha256(pre).digest() if algo == 0 else \
            (K.keccak256(pre) if algo == 1 else hashlib.sha3_256(pre).digest())
        assert d[i].tobytes() == want, (i, t)


@pytest.mark.gpu
@pytest.mark.parametrize("algo", [0, 1, 2])
def test_gpu_variable_length_strings(verifier, algo):
    import torch
    from hyperdrive_amd.digest import hash_bytes_device
    rng = random.Random(20 + algo)
    lens = LENGTHS + [rng.randrange(0, 700) for _ in range(300)]
    rng.shuffle(lens)
    # an odd leading pad so most strings start unaligned
    blobs = [bytes(rng.randrange(256) for _ in range(n)) for n in lens]
    data = b"\x5a" * 3 + b"".join(blobs)
    offs = [3]
    for x in blobs:
        offs.append(offs[-1] + len(x))
    dd = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    do = torch.tensor(offs, dtype=torch.int64).cuda()
    out = hash_bytes_device(verifier, algo, dd, do).cpu().numpy()
    f = {0: lambda x: hashlib.sha256(x).digest(), 1: K.keccak256, 2: lambda x: hashlib.sha3_256(x).digest()}[algo]
    for i, x in enumerate(blobs):
        assert out[i].tobytes() == f(x), (i, len(x))


@pytest.mark.gpu
def test_gpu_verify_over_sha256_lane_equals_verify(verifier, oracle):
    """hd_verify_batch_digest_device over the SHA-256 lane's digests gives the
    verdicts, signatories and signer indices of hd_verify_batch_device on the
    adversarial mix (C5 classes)."""
    import torch
    from hyperdrive_amd.device import DeviceBatch, generate
    from hyperdrive_amd.digest import SHA256, digest_device, verify_digest_device
    S, n = 100, 20000
    db, sigs, _ = generate(verifier, 0, n, S, adv_pct=30, start=12345)
    verifier.set_signatories(sigs)
    dev = db.height.device
    v1 = torch.empty(n, dtype=torch.uint8, device=dev)
    v2 = torch.empty(n, dtype=torch.uint8, device=dev)
    r1 = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    r2 = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    s1 = torch.empty(n, dtype=torch.int32, device=dev)
    s2 = torch.empty(n, dtype=torch.int32, device=dev)
    from hyperdrive_amd.device import work_stream
    ws = work_stream(dev)
    cs = db.c_struct()
    verifier.verify_batch_device(cs, v1.data_ptr(), r1.data_ptr(), s1.data_ptr(), None, ws.cuda_stream)
    dg = digest_device(verifier, SHA256, db, stream=ws)
    verify_digest_device(verifier, db, dg, v2.data_ptr(), r2.data_ptr(), s2.data_ptr(), stream=ws)
    ws.synchronize()
    assert torch.equal(v1, v2) and torch.equal(r1, r2) and torch.equal(s1, s2)
    assert 0 < int((v1 == 0).sum()) < n


@pytest.mark.gpu
def test_gpu_verify_signatures_over_keccak_digests(verifier, oracle):
    """Messages signed over their Keccak-256 preimage digest verify VALID
    through the Keccak lane + hd_verify_batch_digest_device, and fail with
    SIGNATORY_MISMATCH through the SHA-256 path (the reference's digest)."""
    import torch
    from hyperdrive_amd.device import DeviceBatch, work_stream
    from hyperdrive_amd.digest import KECCAK256, digest_device, verify_digest_device
    from hyperdrive_amd.verify import Batch
    keys = oracle.KeyCache()
    S, n = 5, 40
    rng = random.Random(9)
    rows = []
    for i in range(n):
        t = 1 + i % 3
        h, r, vr = 1 + i // 3, rng.randrange(4), rng.randrange(-1, 3)
        val = bytes(rng.randrange(256) for _ in range(32))
        signer = i % S
        dig = K.keccak256(K.preimage(t, h, r, vr, val))
        sig = oracle.sign(keys.sk(signer), dig)
        rows.append((t, h, r, vr, val, keys.signatory(signer), sig))
    b = Batch.from_lists(*[[x[k] for x in rows] for k in range(7)])
    verifier.set_signatories(np.frombuffer(b"".join(keys.signatory(k) for k in range(S)), np.uint8).reshape(S, 32))
    db = DeviceBatch.from_host(b)
    dev = db.height.device
    ws = work_stream(dev)
    vk = torch.empty(n, dtype=torch.uint8, device=dev)
    vs = torch.empty(n, dtype=torch.uint8, device=dev)
    dg = digest_device(verifier, KECCAK256, db, stream=ws)
    verify_digest_device(verifier, db, dg, vk.data_ptr(), stream=ws)
    verifier.verify_batch_device(db.c_struct(), vs.data_ptr(), None, None, None, ws.cuda_stream)
    ws.synchronize()
    assert vk.cpu().tolist() == [0] * n
    assert vs.cpu().tolist() == [5] * n
