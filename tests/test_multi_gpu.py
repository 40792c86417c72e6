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
            rows, counts = route_candidates(v, sub.c_struct(), bits.data_ptr() + 4 * (lo // 32), lo, world, 0)
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
            rb, gidx = unroute(v, recv, 0)
            local = tally_routed_device(v, rb, gidx, 0, tally_out(v, n, pinned=True), "cpu")
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
