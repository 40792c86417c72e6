"""Multi-rank sharding on CPU: world_size 2 (and 3) gloo process groups run the
shard/all-gather logic of the multi-GPU path on oracle-verified bitmaps and
reproduce the single-rank bitmap and tally exactly; the partitioned tally --
each rank tallies only the rounds hd_tally_partition_of gives it, the packed
count tables are all-gathered and merged (shard.gather_tally) -- equals the
single-rank tally rows."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from hyperdrive_amd.shard import gather_bitmaps, gather_bitmaps_async, gather_tally, partition_of, shard_range


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_range_covers_and_aligns():
    for n in [0, 1, 31, 32, 33, 1000, 1 << 20, (1 << 20) + 17]:
        for world in [1, 2, 3, 4, 8]:
            ranges = [shard_range(n, r, world) for r in range(world)]
            assert ranges[0][0] == 0 and ranges[-1][1] == n
            for (lo, hi), (lo2, _) in zip(ranges, ranges[1:]):
                assert hi == lo2 and ((hi - lo) % 32 == 0 or hi == n)   # word-aligned unless it ends the batch
    with pytest.raises(ValueError):
        shard_range(10, 2, 2)


def _bits_of(verdicts):
    v = np.asarray(verdicts)
    bits = np.packbits((v == 0).astype(np.uint8), bitorder="little")
    bits = np.pad(bits, (0, (-len(bits)) % 4))
    return bits.view(np.uint32)


def _worker(rank, world, port, verdicts, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = len(verdicts)
    lo, hi = shard_range(n, rank, world)
    local = torch.from_numpy(_bits_of(verdicts[lo:hi]).view(np.int32).copy())
    full = gather_bitmaps(local, n, world)
    # the bench's asynchronous form: over gloo it gathers at once (work None)
    full2, work = gather_bitmaps_async(local, n, world)
    assert work is None and torch.equal(full, full2)
    # a second communicator (the bench's tally exchange group) works beside the default one
    g2 = dist.new_group(backend="gloo")
    full3 = gather_bitmaps(local, n, world, group=g2)
    assert torch.equal(full, full3)
    out_q.put((rank, full.numpy().view(np.uint32).tolist()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 1000), (3, 1000), (2, 64)])
def test_gloo_bitmap_allgather_matches_single_rank(oracle, world, n):
    rng = np.random.default_rng(world * 1000 + n)
    verdicts = rng.choice([0, 0, 0, 5, 6, 2], size=n).tolist()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, verdicts, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = _bits_of(verdicts)[: (n + 31) // 32].tolist()
    for r in range(world):
        assert res[r] == want


def test_sharded_tally_equals_global(oracle):
    """The tally of the whole batch from gathered per-shard verdicts equals the
    single-rank tally (first-wins across shard boundaries is global)."""
    from tally_cases import scenarios
    sc = [s for s in scenarios() if s.name == "random_mix"][0]
    verdicts = [0 if i % 7 else 5 for i in range(len(sc.b))]
    full = oracle.tally(sc.b, verdicts)
    world = 3
    gathered = []
    for r in range(world):
        lo, hi = shard_range(len(verdicts), r, world)
        gathered += verdicts[lo:hi]
    assert oracle.tally(sc.b, gathered) == full


def tally_rows(b, verdicts, part=0, nparts=1):
    """Packed tally rows (shard.COUNT_COLS / HR_COLS) restated from the
    first-wins rule (process.go:823-892) over the candidates of one partition:
    a round's rep is its first candidate, a value group's rep its first
    winner, rows in rep order."""
    hr, cnt, seen = {}, {}, set()
    for i in range(len(b)):
        t, h, r = b.mtype[i], b.height[i], b.round[i]
        if verdicts[i] != 0 or t not in (2, 3) or partition_of(h, r, nparts) != part:
            continue
        g = hr.setdefault((h, r), {"rep": i, 2: 0, 3: 0, "any": set()})
        key = (h, r, t, b.frm[i])
        if key in seen:
            continue                                   # first wins
        seen.add(key)
        g[t] += 1
        g["any"].add(b.frm[i])
        c = cnt.setdefault((h, r, t, b.value[i]), [i, 0])
        c[1] += 1
    counts = sorted([h, r, t, c[0], c[1]] for (h, r, t, _), c in cnt.items())
    counts.sort(key=lambda row: row[3])
    hrs = sorted(([h, r, g[2], g[3], len(g["any"]), g["rep"]] for (h, r), g in hr.items()), key=lambda row: row[5])
    return {"counts": np.array(counts, np.int64).reshape(-1, 5), "hr": np.array(hrs, np.int64).reshape(-1, 6)}


def test_tally_rows_restatement_matches_oracle(oracle):
    """The row restatement above agrees with the oracle's tally."""
    from tally_cases import scenarios
    sc = [s for s in scenarios() if s.name == "random_mix"][0]
    verdicts = [0 if i % 7 else 5 for i in range(len(sc.b))]
    t = oracle.tally(sc.b, verdicts)
    rows = tally_rows(sc.b, verdicts)
    assert {(h, r, ty, sc.b.value[rep]): n for h, r, ty, rep, n in rows["counts"].tolist()} == t.count
    assert {(h, r): a for h, r, _, _, a, _ in rows["hr"].tolist()} == t.distinct_any


def _tally_worker(rank, world, port, out_q):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__))))
    from tally_cases import scenarios
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sc = [s for s in scenarios() if s.name == "random_mix"][0]
    verdicts = [0 if i % 7 else 5 for i in range(len(sc.b))]
    local = tally_rows(sc.b, verdicts, rank, world)
    merged = gather_tally(local, world)
    # the RCCL ranks' form (rows as tensors, exchange and merge in torch),
    # here on CPU tensors over gloo
    import torch
    from hyperdrive_amd.shard import gather_tally_device
    dev = gather_tally_device({k: torch.from_numpy(v) for k, v in local.items()}, world)
    assert dev["counts"].tolist() == merged["counts"].tolist() and dev["hr"].tolist() == merged["hr"].tolist()
    out_q.put((rank, merged["counts"].tolist(), merged["hr"].tolist(), len(local["hr"])))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_partitioned_tally_equals_single_rank(world):
    from tally_cases import scenarios
    sc = [s for s in scenarios() if s.name == "random_mix"][0]
    verdicts = [0 if i % 7 else 5 for i in range(len(sc.b))]
    want = tally_rows(sc.b, verdicts)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_tally_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, counts, hrs, n_local in res:
        assert counts == want["counts"].tolist() and hrs == want["hr"].tolist()
        assert 0 < n_local < len(want["hr"])             # every rank tallied a strict share of the rounds


# ---- routed tally (the C4 data path: every rank holds only its shard) -------
ROW = 64


def route_rows_np(b, verdicts, lo, hi, nparts, adm_sorted, rounds=None):
    """Restatement of hd_route_candidates_device (include/hd_verify.h) for the
    shard [lo, hi) of an oracle batch: 64-byte rows (h, r: int64 LE; value:
    32 B; global index: u32 LE; admitted sorted index << 8 | type: u32 LE;
    8 zero bytes), grouped by owner, index order inside a group.  rounds (a
    set of (h, r)): hd_route_candidates_listed_device, only those rounds."""
    groups = [[] for _ in range(nparts)]
    index = {a: k for k, a in enumerate(adm_sorted)}
    for i in range(lo, hi):
        t = b.mtype[i]
        if verdicts[i] != 0 or t not in (2, 3):
            continue
        if rounds is not None and (b.height[i], b.round[i]) not in rounds:
            continue
        o = partition_of(b.height[i], b.round[i], nparts)
        row = (int(b.height[i]).to_bytes(8, "little", signed=True) + int(b.round[i]).to_bytes(8, "little", signed=True)
               + b.value[i] + int(i).to_bytes(4, "little") + ((index[b.frm[i]] << 8) | t).to_bytes(4, "little")
               + bytes(8))
        groups[o].append(row)
    counts = [len(g) for g in groups]
    rows = np.frombuffer(b"".join(b"".join(g) for g in groups), np.uint8).reshape(-1, ROW).copy()
    return rows, counts


def unroute_np(rows, adm_sorted):
    """Restatement of hd_unroute_device: rows -> (type, h, r, value, from, gidx) lists."""
    out = []
    for row in rows:
        r = bytes(row)
        st = int.from_bytes(r[52:56], "little")
        out.append((st & 0xFF, int.from_bytes(r[0:8], "little", signed=True), int.from_bytes(r[8:16], "little",
                                                                                             signed=True),
                    r[16:48], adm_sorted[st >> 8], int.from_bytes(r[48:52], "little")))
    return out


class _RB:
    """The oracle-batch face tally_rows reads."""

    def __init__(self, rows):
        self.mtype = [x[0] for x in rows]
        self.height = [x[1] for x in rows]
        self.round = [x[2] for x in rows]
        self.value = [x[3] for x in rows]
        self.frm = [x[4] for x in rows]

    def __len__(self):
        return len(self.mtype)


def routed_tally_rows(rows, adm_sorted):
    """The owner's tally of its received rows, reps mapped to global indices."""
    got = unroute_np(rows, adm_sorted)
    t = tally_rows(_RB(got), [0] * len(got))
    g = np.array([x[5] for x in got], np.int64)
    for key, col in (("counts", 3), ("hr", 5)):
        if len(t[key]):
            t[key][:, col] = g[t[key][:, col]]
    return t


def _routed_worker(rank, world, port, out_q):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__))))
    from tally_cases import scenarios
    from hyperdrive_amd.shard import exchange_routed, gather_tally_device
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sc = [s for s in scenarios() if s.name == "random_mix"][0]
    verdicts = [0 if i % 7 else 5 for i in range(len(sc.b))]
    adm = sorted(set(sc.b.frm))
    lo, hi = shard_range(len(sc.b), rank, world)
    rows, counts = route_rows_np(sc.b, verdicts, lo, hi, world, adm)
    recv = exchange_routed(torch.from_numpy(rows), counts, world)
    local = routed_tally_rows(recv.numpy(), adm)
    merged = gather_tally_device({k: torch.from_numpy(v) for k, v in local.items()}, world)
    out_q.put((rank, merged["counts"].tolist(), merged["hr"].tolist(), int(recv.shape[0]), sum(counts)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_routed_tally_equals_single_rank(world):
    """Each rank routes only its shard's candidates to the owners of their
    rounds (one all-to-all of the counts, one of the rows: shard.
    exchange_routed), every owner tallies what it received, the owners'
    tables are all-gathered and merged: the single-rank tally, row for row."""
    from tally_cases import scenarios
    sc = [s for s in scenarios() if s.name == "random_mix"][0]
    verdicts = [0 if i % 7 else 5 for i in range(len(sc.b))]
    want = tally_rows(sc.b, verdicts)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_routed_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    n_cand = sum(1 for i in range(len(sc.b)) if verdicts[i] == 0 and sc.b.mtype[i] in (2, 3))
    assert sum(r[3] for r in res) == n_cand == sum(r[4] for r in res)   # every candidate reached one owner
    for rank, counts, hrs, n_in, n_out in res:
        assert counts == want["counts"].tolist() and hrs == want["hr"].tolist()


# ---- local tallies + shared rounds only (the default N > 1 exchange) ------
class _Shard:
    """Rows lo .. hi - 1 of an oracle batch, indexed from 0."""

    def __init__(self, b, lo, hi):
        self.mtype, self.height, self.round = b.mtype[lo:hi], b.height[lo:hi], b.round[lo:hi]
        self.value, self.frm = b.value[lo:hi], b.frm[lo:hi]

    def __len__(self):
        return len(self.mtype)


def local_tally_rows(b, verdicts, lo, hi):
    """A rank's tally of its own shard (hd_tally_device_bitmap on the shard),
    reps moved to global indices."""
    t = tally_rows(_Shard(b, lo, hi), verdicts[lo:hi])
    for key, col in (("counts", 3), ("hr", 5)):
        if len(t[key]):
            t[key][:, col] += lo
    return t


def _case(name):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    if name == "random_mix":
        from tally_cases import scenarios
        sc = [s for s in scenarios() if s.name == "random_mix"][0]
        return sc.b, [0 if i % 7 else 5 for i in range(len(sc.b))]
    # heights in index order (the C2 / C4 stream): only rounds cut by a shard
    # boundary are shared; a few duplicates and double votes straddle them
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    import hashlib
    import hd_pyoracle as O
    S = 10                                      # the C2 layout (hd_gen.h kind 0), unsigned: the tally reads no signatures
    b = O.Batch()
    for i in range(600):
        h = 1 + i // (2 * S)
        b.append(2 + (i // S) % 2, h, 0, -1, O.canonical_value(h, 0),
                 hashlib.sha256(b"signer" + bytes([i % S])).digest(), bytes(65))
    # copies of earlier votes just past the shard boundaries (320 for two
    # ranks, 224 and 448 for three), one with a conflicting value (a double
    # vote), and one inside a shard
    for dst, src in ((321, 318), (322, 316), (226, 219), (450, 445), (95, 88)):
        for f in ("mtype", "height", "round", "value", "frm"):
            getattr(b, f)[dst] = getattr(b, f)[src]
    b.value[322] = bytes(32)
    return b, [0 if i % 11 else 6 for i in range(len(b))]


def _hybrid_worker(rank, world, port, name, out_q):
    from hyperdrive_amd.shard import drop_rounds, exchange_routed, gather_tally_device, shared_rounds
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    b, verdicts = _case(name)
    adm = sorted(set(b.frm))
    lo, hi = shard_range(len(b), rank, world)
    local = local_tally_rows(b, verdicts, lo, hi)
    shared = shared_rounds(torch.from_numpy(local["hr"][:, :2].copy()), world)
    rows, counts = route_rows_np(b, verdicts, lo, hi, world, adm, rounds={tuple(x) for x in shared.tolist()})
    recv = exchange_routed(torch.from_numpy(rows), counts, world)
    own = routed_tally_rows(recv.numpy(), adm)
    mine = {k: torch.cat([drop_rounds(torch.from_numpy(local[k]), shared), torch.from_numpy(own[k])])
            for k in ("counts", "hr")}
    merged = gather_tally_device(mine, world)
    out_q.put((rank, merged["counts"].tolist(), merged["hr"].tolist(), sum(counts), len(shared)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("name", ["random_mix", "height_order"])
@pytest.mark.parametrize("world", [2, 3])
def test_gloo_local_tally_plus_shared_rounds_equals_single_rank(world, name):
    """The default N > 1 tally: each rank tallies its own shard, the ranks
    all-gather their round sets (shard.shared_rounds), only the candidates of
    rounds present in more than one shard are routed to their owners
    (hd_route_candidates_listed_device, restated), each rank keeps its local
    rows of the other rounds (shard.drop_rounds) plus the shared rounds it
    owns, and the merged tables equal the single-rank tally row for row --
    with duplicates and a double vote straddling shard boundaries.  In height
    order only the boundary rounds move."""
    b, verdicts = _case(name)
    want = tally_rows(b, verdicts)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_hybrid_worker, args=(r, world, port, name, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, counts, hrs, routed, n_shared in res:
        assert counts == want["counts"].tolist() and hrs == want["hr"].tolist()
    n_cand = sum(1 for i in range(len(b)) if verdicts[i] == 0 and b.mtype[i] in (2, 3))
    routed = sum(r[3] for r in res)
    assert res[0][4] >= 1 and 0 < routed
    if name == "height_order":
        # boundary rounds only: the one a boundary cuts, and one a copied vote reaches
        assert res[0][4] <= 2 * (world - 1) and routed <= 21 * res[0][4] < n_cand


# ---- round ranges (the bench's per-step N > 1 exchange) --------------------
def test_round_ranges_and_masks():
    from hyperdrive_amd.shard import (EMPTY_RANGE, drop_pairs_rows, pairs_isin, ranges_overlap, round_range,
                                      routed_round_mask)
    assert round_range(np.array([], np.int64), np.array([], np.int64)) == EMPTY_RANGE
    assert round_range(np.array([5, 3, 3, 7, 7]), np.array([1, 4, 2, 0, 9])) == (3, 2, 7, 9)
    big = np.iinfo(np.int64).max
    assert round_range(np.array([big, -big]), np.array([-1, 3])) == (-big, 3, big, -1)
    r = np.array([[1, 0, 5, 3], [5, 3, 9, 0], list(EMPTY_RANGE), [20, 0, 30, 0]], np.int64)
    assert ranges_overlap(r)                                       # (5, 3) is in both of the first two
    assert not ranges_overlap(r[[0, 2, 3]])
    assert not ranges_overlap(np.array([[1, 0, 5, 2], [5, 3, 9, 0]], np.int64))   # (5, 2) < (5, 3)
    h, rr = np.array([1, 5, 5, 4]), np.array([0, 3, 2, 7])
    assert routed_round_mask(h, rr, r, 0).tolist() == [False, True, False, False]
    assert not routed_round_mask(h, rr, r[[0]], 0).any()
    rows = np.array([[1, 0, 2], [5, 3, 2], [5, 3, 3], [4, 7, 2]], np.int64)
    assert drop_pairs_rows(rows, np.array([5]), np.array([3])).tolist() == [[1, 0, 2], [4, 7, 2]]
    # the vectorised (> 8 pairs) and the set (spans past 32 bits) forms agree with a set lookup
    rng = np.random.default_rng(3)
    for span in (1000, 1 << 40):
        hh = rng.integers(-span, span, 5000)
        r2 = rng.integers(0, 4, 5000)
        ph, pr = hh[:40].copy(), r2[:40].copy()
        want = {(a, b) for a, b in zip(ph.tolist(), pr.tolist())}
        got = pairs_isin(hh, r2, ph, pr)
        assert got.tolist() == [(a, b) in want for a, b in zip(hh.tolist(), r2.tolist())]


def _range_worker(rank, world, port, name, empty, out_q):
    from hyperdrive_amd.shard import (drop_pairs_rows, exchange_ranges, exchange_routed, gather_tally_device,
                                      ranges_overlap, round_range, routed_round_mask)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    b, verdicts = _case(name)
    if empty is not None:                       # a shard with no candidate at all (an empty range)
        lo_e, hi_e = shard_range(len(b), empty, world)
        verdicts = [5 if lo_e <= i < hi_e else v for i, v in enumerate(verdicts)]
    adm = sorted(set(b.frm))
    lo, hi = shard_range(len(b), rank, world)
    local = local_tally_rows(b, verdicts, lo, hi)
    hh, hr = local["hr"][:, 0], local["hr"][:, 1]
    ranges = exchange_ranges(round_range(hh, hr), world)
    mine, routed, n_rounds = local, 0, 0
    if ranges_overlap(ranges):
        m = routed_round_mask(hh, hr, ranges, rank)
        n_rounds = int(m.sum())
        rows, counts = route_rows_np(b, verdicts, lo, hi, world, adm, rounds=set(zip(hh[m].tolist(), hr[m].tolist())))
        recv = exchange_routed(torch.from_numpy(rows), counts, world)
        own = routed_tally_rows(recv.numpy(), adm)
        mine = {"counts": np.concatenate([drop_pairs_rows(local["counts"], hh[m], hr[m]), own["counts"]]),
                "hr": np.concatenate([local["hr"][~m], own["hr"]])}
        routed = sum(counts)
    merged = gather_tally_device({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in mine.items()}, world)
    out_q.put((rank, merged["counts"].tolist(), merged["hr"].tolist(), routed, n_rounds, len(mine["hr"])))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("name,world,empty", [("random_mix", 2, None), ("height_order", 2, None),
                                              ("random_mix", 3, None), ("height_order", 3, None),
                                              ("height_order", 3, 1), ("height_order", 4, 3)])
def test_gloo_round_ranges_tally_equals_single_rank(name, world, empty):
    """The bench's per-step N > 1 tally: each rank tallies its shard, the
    ranks all-gather only their (height, round) ranges, a rank routes exactly
    its rounds inside another rank's range (hd_route_candidates_listed_device,
    restated) to their owners, keeps the rest, and adds the routed rounds it
    owns.  The ranks' rows are disjoint and, merged, equal the single-rank
    tally row for row -- with duplicates and a double vote straddling shard
    boundaries, shards in random order (most rounds routed), and a shard with
    no candidate (an empty range).  In height order only boundary rounds move."""
    b, verdicts = _case(name)
    if empty is not None:
        lo_e, hi_e = shard_range(len(b), empty, world)
        verdicts = [5 if lo_e <= i < hi_e else v for i, v in enumerate(verdicts)]
    want = tally_rows(b, verdicts)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_range_worker, args=(r, world, port, name, empty, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, counts, hrs, routed, n_rounds, n_mine in res:
        assert counts == want["counts"].tolist() and hrs == want["hr"].tolist()
    assert sum(r[5] for r in res) == len(want["hr"])                # every round tallied by exactly one rank
    if name == "height_order":
        assert sum(r[4] for r in res) <= 3 * (world - 1)            # boundary rounds only
        # (with 3 ranks an empty middle shard leaves no two neighbours to share a round)
        assert (sum(r[4] for r in res) > 0) == ((world, empty) != (3, 1))
