"""The C-ABI multi-GPU path (include/hd_verify.h hd_multi_*,
hyperdrive_amd/multi.py) against the single-context path on the same batches:
verdicts, recovered signatories, the valid bitmap and the merged partitioned
tally are identical.  On a one-GPU box the device list [0] runs the RCCL
exchange (one rank) and [0, 0] / [0, 0, 0] run the copy exchange between
contexts sharing the GPU; an 8-GPU node runs the same code with one rank per
device."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _same(a, b):
    ra, ta = a
    rb, tb = b
    assert ra.verdict.tolist() == rb.verdict.tolist()
    assert ra.recovered.tobytes() == rb.recovered.tobytes()
    assert ra.valid_bitmap.tolist() == rb.valid_bitmap.tolist()
    assert ta.count == tb.count and ta.distinct == tb.distinct and ta.distinct_any == tb.distinct_any
    assert ta.dup.tolist() == tb.dup.tolist()


@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0]])
@pytest.mark.parametrize("kind,n,S,adv", [(0, 65536 + 17, 100, 30), (1, 128064, 1000, 10), (0, 37, 7, 50)])
def test_multi_equals_single(gpu, devices, kind, n, S, adv):
    from hyperdrive_amd.device import generate
    from hyperdrive_amd.multi import MultiVerifier
    v = gpu.Verifier(0)
    ks = v.gen_keys(S)
    v.set_signatories(ks[0])
    db, _, _ = generate(v, kind, n, S, adv, keys=ks)
    hb = db.to_host()
    single = v.process_batch(hb)
    m = MultiVerifier(devices)
    try:
        assert m.uses_rccl == (len(set(devices)) == len(devices))
        m.set_signatories(ks[0])
        for rnd in range(2):                   # pass 2: the per-device known-key tables
            _same(m.process_batch(hb), single)
        assert m.fastpath_stats(0)[0] > 0
    finally:
        m.close()
        v.close()


def test_multi_empty_and_errors(gpu):
    from hyperdrive_amd import _lib
    from hyperdrive_amd.multi import MultiVerifier
    from hyperdrive_amd.verify import Batch
    with pytest.raises(_lib.HDError):
        MultiVerifier([99])
    m = MultiVerifier([0, 0])
    e = Batch(np.zeros(0, np.uint8), np.zeros(0, np.int64), np.zeros(0, np.int64), None,
              np.zeros((0, 32), np.uint8), np.zeros((0, 32), np.uint8), np.zeros((0, 65), np.uint8))
    res, tal = m.process_batch(e)
    assert len(res.verdict) == 0 and tal.count == {}
    m.close()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_routed_kernels_match_restatement(gpu, world):
    """hd_route_candidates_device / hd_unroute_device / hd_tally_routed_device
    (the C4 data path) on one GPU, every rank's shard in turn: the route rows
    are byte-identical to the restatement (tests/test_multi_rank.py
    route_rows_np), the rebuilt batches and global indices to unroute_np, each
    owner's tally to its restated rows, and the owners' merged tables to the
    single-context tally of the whole batch."""
    import torch
    from test_multi_rank import route_rows_np, routed_tally_rows, tally_rows
    from util import from_np
    from hyperdrive_amd.device import DeviceBatch, generate
    from hyperdrive_amd.shard import (merge_tally_parts, route_candidates, shard_range, tally_out,
                                      tally_routed_device, unroute)
    v = gpu.Verifier(0)
    # the library's kernels on torch's current stream: the rows it writes are
    # read by torch copies, and the received rows torch.cat builds are read
    # by the library (on the context's own stream they would race)
    cs = torch.cuda.current_stream().cuda_stream
    try:
        S, n = 50, 20_000 + 13
        ks = v.gen_keys(S)
        v.set_signatories(ks[0])
        db, _, _ = generate(v, 0, n, S, 30, keys=ks, start=99)
        hb = db.to_host()
        res, whole = v.process_batch(hb)
        ob = from_np(hb)
        verdicts = res.verdict.tolist()
        adm = sorted(bytes(x) for x in ks[0])
        bits = torch.from_numpy(res.valid_bitmap.view(np.int32).copy()).cuda()
        sent = {}
        for k in range(world):
            lo, hi = shard_range(n, k, world)
            sub = DeviceBatch(hi - lo, db.type[lo:hi], db.height[lo:hi], db.round[lo:hi], db.valid_round[lo:hi],
                              db.value[lo:hi], db.frm[lo:hi], db.sig[lo:hi])
            rows, counts = route_candidates(v, sub.c_struct(), bits.data_ptr() + 4 * (lo // 32), lo, world, cs)
            want, want_counts = route_rows_np(ob, verdicts, lo, hi, world, adm)
            assert counts == want_counts
            got = rows[: sum(counts)].cpu().numpy()
            assert got.tobytes() == want.tobytes()
            off = np.concatenate([[0], np.cumsum(counts)])
            for o in range(world):
                sent[(k, o)] = rows[off[o]: off[o + 1]]
        parts = []
        for o in range(world):
            recv = torch.cat([sent[(k, o)] for k in range(world)]).contiguous()
            rb, gidx = unroute(v, recv, cs)
            local = tally_routed_device(v, rb, gidx, cs, tally_out(v, n, pinned=True), "cpu")
            want = routed_tally_rows(recv.cpu().numpy(), adm)
            assert local["counts"].tolist() == want["counts"].tolist()
            assert local["hr"].tolist() == want["hr"].tolist()
            parts.append({k: t.numpy() for k, t in local.items()})
        merged = merge_tally_parts(parts)
        single = tally_rows(ob, verdicts)
        assert merged["counts"].tolist() == single["counts"].tolist()
        assert merged["hr"].tolist() == single["hr"].tolist()
        assert sum(merged["counts"][:, 4].tolist()) == sum(whole.count.values())
    finally:
        v.close()


def test_route_refuses_candidates_outside_the_set(gpu):
    """A VALID candidate whose From left the admitted set after verification
    cannot be named by a route row (rows carry the admitted index), so
    hd_route_candidates_device refuses the batch (HD_EINVAL, with the count in
    the context's last error) instead of tallying it under a synthetic From;
    with the set restored the same call routes every candidate."""
    import torch
    from hyperdrive_amd import _lib
    from hyperdrive_amd.device import generate
    from hyperdrive_amd.shard import route_candidates
    v = gpu.Verifier(0)
    try:
        S, n = 20, 4096
        ks = v.gen_keys(S)
        v.set_signatories(ks[0])
        db, _, _ = generate(v, 0, n, S, 0, keys=ks)
        res = v.verify_batch(db.to_host())
        bits = torch.from_numpy(res.valid_bitmap.view(np.int32).copy()).cuda()
        cs = torch.cuda.current_stream().cuda_stream   # ordered after the bitmap's upload
        v.set_signatories(ks[0][: S // 2])          # half the signers leave
        with pytest.raises(_lib.HDError) as e:
            route_candidates(v, db.c_struct(), bits.data_ptr(), 0, 3, cs)
        assert e.value.code == _lib.HD_EINVAL and "not in the current admitted set" in str(e.value)
        v.set_signatories(ks[0])
        _, counts = route_candidates(v, db.c_struct(), bits.data_ptr(), 0, 3, cs)
        assert sum(counts) == int((res.verdict == 0).sum())
    finally:
        v.close()
