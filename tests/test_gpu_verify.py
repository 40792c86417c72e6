"""GPU parity: k_verify (through the C ABI) against the oracle, and the GPU
generator against the oracle's workload definition."""
import numpy as np
import pytest

from util import from_np, to_np

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def verifier(gpu):
    v = gpu.Verifier(0)
    yield v
    v.close()


@pytest.mark.parametrize("compressed", [True, False])
@pytest.mark.parametrize("kind,S,n,adv", [(0, 10, 300, 60), (1, 7, 150, 40), (0, 100, 257, 30), (1, 1000, 2001 + 5, 10)])
def test_verify_parity_vs_oracle(gpu, oracle, kind, S, n, adv, compressed):
    v = gpu.Verifier(0, compressed=compressed)
    keys = oracle.KeyCache(compressed)
    ob, _ = oracle.gen_batch(kind, min(n, 400), S, adv, keys=keys) if S < 1000 else _rounds_head(oracle, keys, n)
    adm = oracle.admitted_set(S, keys)
    v.set_signatories(adm)
    res = v.verify_batch(to_np(ob))
    vs, recs = oracle.verify_batch(ob, adm, compressed)
    assert res.verdict.tolist() == vs
    assert res.recovered.tobytes() == b"".join(recs)
    bits = np.unpackbits(res.valid_bitmap.view(np.uint8), bitorder="little")[: len(ob)]
    assert bits.tolist() == [int(x == oracle.VALID) for x in vs]
    v.close()


def _rounds_head(oracle, keys, n):
    # C3 shape (1000 signers) without signing 2001 messages in Python: the
    # first 40 messages of round 0 plus a few from round 1
    b1, c1 = oracle.gen_batch(oracle.GEN_ROUNDS, 40, 1000, 10, keys=keys)
    b2, c2 = oracle.gen_batch(oracle.GEN_ROUNDS, 5, 1000, 10, start=2001, keys=keys)
    for i in range(len(b2)):
        b1.append(b2.mtype[i], b2.height[i], b2.round[i], b2.valid_round[i], b2.value[i], b2.frm[i], b2.sig[i])
    return b1, c1 + c2


@pytest.mark.parametrize("kind,S,n,adv,start", [(0, 10, 300, 60, 0), (1, 7, 150, 40, 0), (0, 100, 64, 30, 999_936)])
def test_gpu_generator_matches_oracle(verifier, oracle, kind, S, n, adv, start):
    from hyperdrive_amd.device import generate
    keys = oracle.KeyCache()
    ks = verifier.gen_keys(S)
    assert ks[0].tobytes() == b"".join(oracle.admitted_set(S, keys))
    db, _, _ = generate(verifier, kind, n, S, adv, start=start, keys=ks)
    hb = db.to_host()
    ob, cls = oracle.gen_batch(kind, n, S, adv, start=start, keys=keys)
    assert hb.type.tolist() == ob.mtype
    assert hb.height.tolist() == ob.height and hb.round.tolist() == ob.round
    assert hb.value.tobytes() == b"".join(ob.value)
    assert hb.frm.tobytes() == b"".join(ob.frm)
    assert hb.sig.tobytes() == b"".join(ob.sig)
    assert db.adv_class.cpu().numpy().tolist() == cls


def test_edge_cases(verifier, oracle):
    keys = oracle.KeyCache()
    adm = oracle.admitted_set(4, keys)
    verifier.set_signatories(adm + adm[:2])          # duplicates in the admitted set are harmless
    empty = to_np(oracle.Batch())
    res = verifier.verify_batch(empty)
    assert len(res.verdict) == 0
    for n in (1, 31, 33, 63, 64, 65, 127):             # ragged sizes around the 32/64 bitmap words
        ob, _ = oracle.gen_batch(oracle.GEN_VOTES, n, 4, 40, keys=keys)
        res = verifier.verify_batch(to_np(ob))
        vs, _ = oracle.verify_batch(ob, adm)
        assert res.verdict.tolist() == vs
        bits = np.unpackbits(res.valid_bitmap.view(np.uint8), bitorder="little")[:n]
        assert bits.tolist() == [int(x == 0) for x in vs]
    ob, _ = oracle.gen_batch(oracle.GEN_VOTES, 20, 4, 0, keys=keys)
    nb = to_np(ob)
    nb.type[[2, 3, 4]] = [0, 4, 200]
    nb.valid_round = None                              # optional field
    res = verifier.verify_batch(nb)
    ref, _ = oracle.verify_batch(from_np(nb), adm)
    assert res.verdict.tolist() == ref
    assert res.verdict[2] == res.verdict[3] == res.verdict[4] == oracle.BAD_TYPE
    verifier.set_signatories([])                       # empty admitted set: nothing is admitted
    res = verifier.verify_batch(to_np(ob))
    assert set(res.verdict.tolist()) == {oracle.NOT_ADMITTED}


def test_full_size_c2_properties(verifier, oracle, coracle):
    """1M messages (BASELINE configs[1]): every honest message must verify to its
    own signer (by construction), the bitmap must agree with the verdicts, and a
    seeded sample must match the C oracle bit for bit."""
    import torch
    from hyperdrive_amd.device import generate
    N, S = 1 << 20, 100
    ks = verifier.gen_keys(S)
    verifier.set_signatories(ks[0])
    db, _, _ = generate(verifier, 0, N, S, 0, keys=ks)
    verdict = torch.empty(N, dtype=torch.uint8, device="cuda")
    signer = torch.empty(N, dtype=torch.int32, device="cuda")
    rec = torch.empty((N, 32), dtype=torch.uint8, device="cuda")
    bm = torch.empty(N // 32, dtype=torch.int32, device="cuda")
    from hyperdrive_amd.device import work_stream
    stream = work_stream().cuda_stream
    verifier.verify_batch_device(db.c_struct(), verdict.data_ptr(), rec.data_ptr(), signer.data_ptr(), bm.data_ptr(),
                                 stream)
    torch.cuda.synchronize()
    assert int((verdict != 0).sum()) == 0
    idx = torch.arange(N, device="cuda", dtype=torch.int64)
    assert bool((signer.long() == idx % S).all())
    assert bool((rec == db.frm).all())
    assert int(bm.view(torch.uint8).cpu().numpy().astype(np.uint8).sum()) == 255 * (N // 8)
    # sample vs the C oracle
    rng = np.random.default_rng(5)
    pick = np.sort(rng.choice(N, 512, replace=False))
    hb = db.to_host()
    from hyperdrive_amd.verify import Batch
    sb = Batch(hb.type[pick], hb.height[pick], hb.round[pick], hb.valid_round[pick], hb.value[pick], hb.frm[pick],
               hb.sig[pick])
    cv, crec = coracle.verify(sb, ks[0], True, threads=8)
    assert cv.tolist() == verdict.cpu().numpy()[pick].tolist()
    assert crec.tobytes() == rec.cpu().numpy()[pick].tobytes()


def test_adversarial_full_mix_vs_c_oracle(verifier, oracle, coracle):
    """C5-style mix: 30 % adversarial across all classes, 64k messages, checked
    message by message against the C oracle."""
    import torch
    from hyperdrive_amd.device import generate
    N, S = 65536, 100
    ks = verifier.gen_keys(S)
    verifier.set_signatories(ks[0])
    db, _, _ = generate(verifier, 0, N, S, 30, keys=ks)
    hb = db.to_host()
    res = verifier.verify_batch(hb)
    cv, crec = coracle.verify(hb, ks[0], True, threads=16)
    assert res.verdict.tolist() == cv.tolist()
    assert res.recovered.tobytes() == crec.tobytes()
    hist = np.bincount(res.verdict, minlength=8)
    assert hist[0] > 0.7 * N and all(hist[k] > 0 for k in range(1, 7))
