"""Multi-GPU sharding of a batch.

One process per GPU (torch.distributed; backend "nccl" is RCCL on ROCm, "gloo"
in the CPU tests).  Verification is embarrassingly parallel per message, so
rank k verifies the contiguous index range ``shard_range(n, k, world)`` of a
batch whose metadata is replicated on every rank; the only exchange is an
all-gather of the per-rank valid bitmaps (n/32 words in total, latency-bound
over xGMI).

The tally: first-wins is per (height, round, type, signer), so a round whose
candidates all sit in one shard is complete there.  Each rank tallies its own
shard; the ranks all-gather their round sets (``shared_rounds``: a few
thousand (height, round) pairs) and only the candidates of rounds present in
more than one shard -- the rounds straddling a shard boundary -- are routed
to the owner of the round (``partition_of``) by one all-to-all
(``route_candidates(rounds=...)`` / ``exchange_routed``).  Each rank keeps
its local rows of the other rounds (``drop_rounds``) plus the rows of the
shared rounds it owns, and the small tables are all-gathered and merged in
first-batch-index order (``gather_tally_device``), which is exactly the
single-GPU tally's output order.  (The older partitioned forms -- every rank
tallying the rounds it owns from a replicated batch, or every candidate
routed to its owner -- stay available.)
"""
from __future__ import annotations

import ctypes
from typing import Dict, List, Tuple

import numpy as np

# rows of a packed tally part (int64 columns)
COUNT_COLS = ("count_height", "count_round", "count_type", "count_rep", "count_n")
HR_COLS = ("hr_height", "hr_round", "hr_prevotes", "hr_precommits", "hr_any", "hr_rep")


def shard_range(n: int, rank: int, world: int, align: int = 32) -> Tuple[int, int]:
    """[lo, hi) of rank's shard: contiguous, bitmap-word aligned (every shard
    but the last is a multiple of ``align`` messages), covering [0, n)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of {world}")
    per = (n + world - 1) // world
    per = (per + align - 1) // align * align
    lo = min(n, rank * per)
    hi = min(n, lo + per)
    return lo, hi


def gather_bitmaps(local_bits, n: int, world: int, group=None):
    """All-gather per-rank valid bitmaps (int32 tensors of shard_len/32 words,
    shard-aligned) into one bitmap of ceil(n/32) words, in rank order.

    Every shard except the last is a whole number of words (shard_range's
    alignment), so the concatenation is exactly the global bitmap."""
    import torch
    import torch.distributed as dist
    if local_bits.is_cuda and dist.get_backend(group) == "gloo":
        # gloo moves host tensors only (CPU rehearsal of the multi-GPU path)
        return gather_bitmaps(local_bits.cpu(), n, world, group).to(local_bits.device)
    per_words = [(shard_range(n, r, world)[1] - shard_range(n, r, world)[0] + 31) // 32 for r in range(world)]
    if len(set(per_words)) == 1:
        out = torch.empty(per_words[0] * world, dtype=local_bits.dtype, device=local_bits.device)
        dist.all_gather_into_tensor(out, local_bits.contiguous(), group=group)
        return out[: (n + 31) // 32]
    # ragged last shard: pad to the largest shard, gather, then trim
    width = max(per_words)
    padded = torch.zeros(width, dtype=local_bits.dtype, device=local_bits.device)
    padded[: local_bits.numel()] = local_bits
    out = torch.empty(width * world, dtype=local_bits.dtype, device=local_bits.device)
    dist.all_gather_into_tensor(out, padded, group=group)
    parts = [out[r * width: r * width + per_words[r]] for r in range(world)]
    return torch.cat(parts)[: (n + 31) // 32]


def gather_bitmaps_async(local_bits, n: int, world: int, group=None):
    """gather_bitmaps without making the calling stream wait: returns
    (bitmap, work).  With RCCL and equal shards the all-gather is issued with
    async_op=True; the consumer calls work.wait() on ITS stream (so the next
    verification on the caller's stream does not wait for the exchange).  Any
    other case gathers synchronously and returns work = None."""
    import torch.distributed as dist
    per_words = {(shard_range(n, r, world)[1] - shard_range(n, r, world)[0] + 31) // 32 for r in range(world)}
    if not local_bits.is_cuda or dist.get_backend(group) != "nccl" or len(per_words) != 1:
        return gather_bitmaps(local_bits, n, world, group), None
    import torch
    out = torch.empty(per_words.pop() * world, dtype=local_bits.dtype, device=local_bits.device)
    work = dist.all_gather_into_tensor(out, local_bits.contiguous(), group=group, async_op=True)
    return out[: (n + 31) // 32], work


def partition_of(height: int, round_: int, nparts: int) -> int:
    """The rank that tallies (height, round) among nparts
    (include/hd_verify.h hd_tally_partition_of; a host function of the
    library, no device needed)."""
    from . import _lib
    return int(_lib.load().hd_tally_partition_of(int(height), int(round_), int(nparts)))


def tally_out(v, n: int, pinned: bool = False):
    """A reusable output struct for tally_part over n messages (no per-message
    dup classification: the partitions' packed rows do not carry it)."""
    t, a = v._tally_struct(n, pinned=pinned)
    t.dup = None
    return t, a


def tally_part(v, dbatch, d_bitmap: int, part: int, nparts: int, stream=None, out=None) -> Dict[str, np.ndarray]:
    """This rank's partition of the tally of a device batch (all messages,
    replicated) given the gathered valid bitmap: the packed rows
    {"counts": [k, 5] int64, "hr": [m, 6] int64} (COUNT_COLS / HR_COLS).
    out: a struct from tally_out, reused across calls."""
    from . import _lib
    lib = _lib.load()
    t, a = out if out is not None else tally_out(v, dbatch.n)
    rc = lib.hd_tally_device_bitmap_part(v.handle, ctypes.byref(dbatch), d_bitmap, part, nparts, ctypes.byref(t),
                                         stream)
    if rc != 0:
        raise _lib.HDError(rc, "hd_tally_device_bitmap_part", lib.hd_ctx_last_error(v.handle).decode())
    return pack_tally(a, t.n_counts, t.n_hr)


def tally_part_device(v, dbatch, d_bitmap: int, part: int, nparts: int, stream, out, device):
    """tally_part, with the packed rows left as int64 tensors on `device`
    ({"counts": [k, 5], "hr": [m, 6]}): the library's outputs (pinned host
    memory, `out` from tally_out(..., pinned=True)) go back up in one copy
    per column, so the exchange and the merge stay on the GPU."""
    import torch
    from . import _lib
    lib = _lib.load()
    t, a = out
    # the previous call's uploads may still be reading the pinned stage that
    # the library is about to overwrite: wait for them first
    prev = getattr(t, "_uploads_done", None)
    if prev is not None:
        prev.synchronize()
    rc = lib.hd_tally_device_bitmap_part(v.handle, ctypes.byref(dbatch), d_bitmap, part, nparts, ctypes.byref(t),
                                         stream)
    if rc != 0:
        raise _lib.HDError(rc, "hd_tally_device_bitmap_part", lib.hd_ctx_last_error(v.handle).decode())

    def rows(cols, k):
        if k == 0:
            return torch.zeros((0, len(cols)), dtype=torch.int64, device=device)
        return torch.stack([torch.from_numpy(a[c][:k].astype(np.int64, copy=False)).to(device, non_blocking=True)
                            for c in cols], 1)
    res = {"counts": rows(COUNT_COLS, t.n_counts), "hr": rows(HR_COLS, t.n_hr)}
    if torch.device(device).type == "cuda":
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(device))
        t._uploads_done = ev
    return res


def gather_tally_device(local, world: int, group=None):
    """gather_tally for RCCL ranks with the rows already on the GPU: sizes
    all-gathered (the only host read), then the rows padded to the largest,
    then the merge -- concatenation and a sort by first batch index -- on
    the device.  Returns the merged int64 tensors on the device."""
    import torch
    import torch.distributed as dist
    dev = local["counts"].device
    if local["counts"].is_cuda and dist.get_backend(group) == "gloo":
        out = gather_tally_device({k: t.cpu() for k, t in local.items()}, world, group)
        return {k: t.to(dev) for k, t in out.items()}
    sizes = torch.tensor([local["counts"].shape[0], local["hr"].shape[0]], dtype=torch.int64, device=dev)
    all_sizes = torch.empty(2 * world, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(all_sizes, sizes, group=group)
    all_sizes = all_sizes.view(world, 2).cpu()
    merged = {}
    for j, (key, cols, rep_col) in enumerate((("counts", 5, 3), ("hr", 6, 5))):
        width = max(1, int(all_sizes[:, j].max()))
        pad = torch.zeros((width, cols), dtype=torch.int64, device=dev)
        pad[: local[key].shape[0]] = local[key]
        out = torch.empty((world * width, cols), dtype=torch.int64, device=dev)
        dist.all_gather_into_tensor(out, pad, group=group)
        keep = (torch.arange(width, device=dev)[None, :] < all_sizes[:, j].to(dev)[:, None]).reshape(-1)
        rows = out[keep]
        merged[key] = rows[torch.argsort(rows[:, rep_col], stable=True)]
    return merged


# ---- the per-step exchange of the bench's N > 1 tally: round ranges --------
# Each rank tallies its own shard (hd_tally_device_bitmap on the shard, rows
# on the host).  A round whose candidates sit in one shard only is complete
# there.  To find the rounds that may not be, the ranks exchange only the
# lexicographic range [min, max] of their (height, round) pairs (one
# all-gather of 4 int64): a round of this rank inside ANOTHER rank's range is
# routed (every candidate of it in this shard goes to the round's owner,
# partition_of); every other round stays local.  A round held by two ranks
# lies inside both ranges, so both route it and its owner sees all of its
# candidates (first-wins per (h, r, type, signer) needs them all,
# process/process.go:823-892); a round routed by one rank only is tallied by
# its owner from that rank's candidates alone -- the same rows.  In height
# order (the C2 / C4 stream) only the rounds a shard boundary cuts fall inside
# a neighbour's range; nothing else moves.  The ranks' final rows are disjoint
# (each round tallied once) and their union is the single-GPU tally: each
# rank holds the rounds it tallied, and merging them (gather_tally_device) is
# the consumer's choice, not a per-step cost.
EMPTY_RANGE = (np.iinfo(np.int64).max, np.iinfo(np.int64).max, np.iinfo(np.int64).min, np.iinfo(np.int64).min)


def round_range(h: np.ndarray, r: np.ndarray) -> Tuple[int, int, int, int]:
    """(hmin, rmin, hmax, rmax): the lexicographic extremes of the pairs
    (h[k], r[k]); EMPTY_RANGE (min > max) for none."""
    if len(h) == 0:
        return EMPTY_RANGE
    h = np.asarray(h, np.int64)
    r = np.asarray(r, np.int64)
    hmin, hmax = int(h.min()), int(h.max())
    return hmin, int(r[h == hmin].min()), hmax, int(r[h == hmax].max())


def _range_empty(g) -> bool:
    return (g[0], g[1]) > (g[2], g[3])


def exchange_ranges(rng, world: int, group=None, device=None) -> np.ndarray:
    """All-gather every rank's round_range: an int64 [world, 4] array on the
    host (one collective, one 32-byte-per-rank read back).  device: where the
    collective runs (CUDA for RCCL; None or a gloo group: the CPU)."""
    import torch
    import torch.distributed as dist
    if device is None or dist.get_backend(group) == "gloo":
        device = "cpu"
    t = torch.tensor(list(rng), dtype=torch.int64, device=device)
    out = torch.empty(4 * world, dtype=torch.int64, device=device)
    dist.all_gather_into_tensor(out, t, group=group)
    return out.view(world, 4).cpu().numpy()


def ranges_overlap(ranges: np.ndarray) -> bool:
    """Whether any two non-empty ranges overlap -- exactly when some rank has a
    round inside another's range (an overlap contains an endpoint of one
    range, and endpoints are rounds), i.e. when any rank routes anything.
    Every rank computes the same answer from the gathered ranges."""
    live = [tuple(int(x) for x in g) for g in ranges if not _range_empty(g)]
    for i in range(len(live)):
        for j in range(i + 1, len(live)):
            a, b = live[i], live[j]
            lo = max((a[0], a[1]), (b[0], b[1]))
            hi = min((a[2], a[3]), (b[2], b[3]))
            if lo <= hi:
                return True
    return False


def routed_round_mask(h: np.ndarray, r: np.ndarray, ranges: np.ndarray, rank: int) -> np.ndarray:
    """Per pair (h[k], r[k]) of this rank: inside some other rank's range."""
    h = np.asarray(h, np.int64)
    r = np.asarray(r, np.int64)
    m = np.zeros(len(h), bool)
    for k, g in enumerate(ranges):
        if k == rank or _range_empty(g):
            continue
        hmin, rmin, hmax, rmax = (int(x) for x in g)
        ge = (h > hmin) | ((h == hmin) & (r >= rmin))
        le = (h < hmax) | ((h == hmax) & (r <= rmax))
        m |= ge & le
    return m


def pairs_isin(h: np.ndarray, r: np.ndarray, ph: np.ndarray, pr: np.ndarray) -> np.ndarray:
    """Per pair (h[k], r[k]): one of the pairs (ph[j], pr[j])."""
    h = np.asarray(h, np.int64)
    r = np.asarray(r, np.int64)
    ph = np.asarray(ph, np.int64)
    pr = np.asarray(pr, np.int64)
    if len(ph) == 0 or len(h) == 0:
        return np.zeros(len(h), bool)
    if len(ph) <= 8:
        m = np.zeros(len(h), bool)
        for a, b in zip(ph.tolist(), pr.tolist()):
            m |= (h == a) & (r == b)
        return m
    # one int64 key per pair when both spans fit 32 bits, else a set lookup
    h0, r0 = min(int(h.min()), int(ph.min())), min(int(r.min()), int(pr.min()))
    h1, r1 = max(int(h.max()), int(ph.max())), max(int(r.max()), int(pr.max()))
    if h1 - h0 < (1 << 31) and r1 - r0 < (1 << 32):
        key = lambda x, y: ((x - h0) << 32) | (y - r0)
        return np.isin(key(h, r), key(ph, pr))
    want = set(zip(ph.tolist(), pr.tolist()))
    return np.fromiter(((a, b) in want for a, b in zip(h.tolist(), r.tolist())), bool, len(h))


def drop_pairs_rows(rows: np.ndarray, ph: np.ndarray, pr: np.ndarray) -> np.ndarray:
    """rows (int64 [m, c], columns 0 and 1 height and round) without those of
    the given pairs."""
    if len(rows) == 0 or len(ph) == 0:
        return rows
    return rows[~pairs_isin(rows[:, 0], rows[:, 1], ph, pr)]


# ---- routed tally (the C4 data path: no replicated batch) -----------------
ROUTE_ROW_BYTES = 64       # include/hd_verify.h HD_ROUTE_ROW_BYTES


def route_candidates(v, dshard, d_bitmap: int, base_index: int, world: int, stream, rows=None, rounds=None):
    """This rank's candidates (VALID Prevotes / Precommits of its shard, global
    index base_index + i) as route rows grouped by the owner of their round
    (hd_route_candidates_device).  Returns (rows uint8 tensor [cap, 64], counts
    list of `world` ints); rows may be passed in for reuse.  rounds: an int64
    [k, 2] CUDA tensor of (height, round) pairs sorted lexicographically
    (shared_rounds): only candidates of those rounds are routed
    (hd_route_candidates_listed_device)."""
    import torch
    from . import _lib
    lib = _lib.load()
    n = dshard.n
    dev = torch.device("cuda", v.device)
    if rows is None or rows.shape[0] < max(n, 1):
        rows = torch.empty((max(n, 1), ROUTE_ROW_BYTES), dtype=torch.uint8, device=dev)
    counts = (ctypes.c_uint32 * world)()
    if rounds is None:
        rc = lib.hd_route_candidates_device(v.handle, ctypes.byref(dshard), d_bitmap, int(base_index), int(world),
                                            rows.data_ptr(), rows.shape[0], counts, stream)
        where = "hd_route_candidates_device"
    else:
        rh = rounds[:, 0].contiguous()
        rr = rounds[:, 1].contiguous()
        k = int(rounds.shape[0])
        rc = lib.hd_route_candidates_listed_device(v.handle, ctypes.byref(dshard), d_bitmap, int(base_index),
                                                   int(world), rh.data_ptr() if k else None,
                                                   rr.data_ptr() if k else None, k, rows.data_ptr(), rows.shape[0],
                                                   counts, stream)
        where = "hd_route_candidates_listed_device"
    if rc != 0:
        raise _lib.HDError(rc, where, lib.hd_ctx_last_error(v.handle).decode())
    return rows, [int(c) for c in counts]


def shared_rounds(local_rounds, world: int, group=None):
    """The (height, round) pairs that occur in more than one rank's shard,
    as an int64 [k, 2] tensor sorted lexicographically, identical on every
    rank.  local_rounds: this rank's distinct rounds ([m, 2] int64, e.g. the
    first two columns of its local tally's hr rows).  One all-gather of the
    sizes and one of the pairs (padded to the largest); torch only, so it runs
    over RCCL on the device and over gloo on the CPU."""
    import torch
    import torch.distributed as dist
    dev = local_rounds.device
    if local_rounds.is_cuda and dist.get_backend(group) == "gloo":
        return shared_rounds(local_rounds.cpu(), world, group).to(dev)
    pairs = local_rounds.to(torch.int64).reshape(-1, 2)
    size = torch.tensor([pairs.shape[0]], dtype=torch.int64, device=dev)
    sizes = torch.empty(world, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(sizes, size, group=group)
    sizes = sizes.cpu().tolist()
    width = max(1, max(sizes))
    pad = torch.zeros((width, 2), dtype=torch.int64, device=dev)
    pad[: pairs.shape[0]] = pairs
    out = torch.empty((world * width, 2), dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(out, pad, group=group)
    keep = (torch.arange(width, device=dev)[None, :] < torch.tensor(sizes, device=dev)[:, None]).reshape(-1)
    allp = out[keep]
    if allp.shape[0] == 0:
        return allp
    # a rank lists each of its rounds once, so a pair seen twice is shared
    uniq, cnt = torch.unique(allp, dim=0, return_counts=True)   # rows sorted lexicographically
    return uniq[cnt > 1].contiguous()


def drop_rounds(rows, rounds):
    """rows (an int64 [m, c] tensor whose first two columns are height and
    round) without those of the given (height, round) pairs."""
    import torch
    if rows.shape[0] == 0 or rounds.shape[0] == 0:
        return rows
    both = torch.cat([rounds.to(rows.device), rows[:, :2]])
    _, inv = torch.unique(both, dim=0, return_inverse=True)
    shared_ids = inv[: rounds.shape[0]]
    mask = ~torch.isin(inv[rounds.shape[0]:], shared_ids)
    return rows[mask]


def exchange_routed(rows, counts, world: int, group=None):
    """All-to-all of the route rows: rank o receives every rank's group o, in
    source-rank order (= global index order).  rows: [>= sum(counts), 64] uint8
    tensor (CUDA for RCCL, CPU for gloo).  Returns the received rows tensor.
    One host read per call: the receive sizes (an all-to-all of the counts)."""
    import torch
    import torch.distributed as dist
    if rows.is_cuda and dist.get_backend(group) == "gloo":
        # gloo moves host tensors only (CPU rehearsal of the multi-GPU path)
        return exchange_routed(rows[: sum(counts)].cpu(), counts, world, group).to(rows.device)
    send = torch.tensor(counts, dtype=torch.int64, device=rows.device)
    recv = torch.empty(world, dtype=torch.int64, device=rows.device)
    dist.all_to_all_single(recv, send, group=group)
    rc = recv.cpu().tolist()
    out = torch.empty((max(sum(rc), 1), ROUTE_ROW_BYTES), dtype=torch.uint8, device=rows.device)
    total = sum(counts)
    dist.all_to_all_single(out[: sum(rc)], rows[:total], output_split_sizes=rc, input_split_sizes=list(counts),
                           group=group)
    return out[: sum(rc)]


def unroute(v, rows, stream):
    """Received route rows -> (DeviceBatch, gidx int32 tensor) (hd_unroute_device)."""
    import torch
    from . import _lib
    from .device import DeviceBatch
    lib = _lib.load()
    m = rows.shape[0]
    db = DeviceBatch.empty(m, str(rows.device))
    gidx = torch.empty(max(m, 1), dtype=torch.int32, device=rows.device)
    if m:
        rc = lib.hd_unroute_device(v.handle, rows.data_ptr(), m, ctypes.byref(db.c_out()), gidx.data_ptr(), stream)
        if rc != 0:
            raise _lib.HDError(rc, "hd_unroute_device", lib.hd_ctx_last_error(v.handle).decode())
    return db, gidx[:m]


def tally_routed_device(v, db, gidx, stream, out, device):
    """The owner's tally of its received candidates (hd_tally_routed_device):
    packed rows {"counts": [k, 5], "hr": [m, 6]} as int64 tensors on `device`,
    reps already global indices.  out: a pinned struct from tally_out."""
    import torch
    from . import _lib
    lib = _lib.load()
    t, a = out
    if db.n == 0:
        return {"counts": torch.zeros((0, 5), dtype=torch.int64, device=device),
                "hr": torch.zeros((0, 6), dtype=torch.int64, device=device)}
    rc = lib.hd_tally_routed_device(v.handle, ctypes.byref(db.c_struct()), gidx.data_ptr(), ctypes.byref(t), stream)
    if rc != 0:
        raise _lib.HDError(rc, "hd_tally_routed_device", lib.hd_ctx_last_error(v.handle).decode())
    packed = pack_tally(a, t.n_counts, t.n_hr)     # host copies of the pinned stage: the next call may reuse it
    return {"counts": torch.from_numpy(packed["counts"]).to(device), "hr": torch.from_numpy(packed["hr"]).to(device)}


def tally_routed_host(v, db, gidx, stream, out) -> Dict[str, np.ndarray]:
    """tally_routed_device with the packed rows left on the host (numpy
    int64 {"counts": [k, 5], "hr": [m, 6]}, reps global indices)."""
    from . import _lib
    lib = _lib.load()
    t, a = out
    if db.n == 0:
        return {"counts": np.zeros((0, 5), np.int64), "hr": np.zeros((0, 6), np.int64)}
    rc = lib.hd_tally_routed_device(v.handle, ctypes.byref(db.c_struct()), gidx.data_ptr(), ctypes.byref(t), stream)
    if rc != 0:
        raise _lib.HDError(rc, "hd_tally_routed_device", lib.hd_ctx_last_error(v.handle).decode())
    return pack_tally(a, t.n_counts, t.n_hr)


def pack_tally(a, n_counts: int, n_hr: int) -> Dict[str, np.ndarray]:
    return {"counts": np.stack([a[c][:n_counts].astype(np.int64) for c in COUNT_COLS], 1).reshape(n_counts, 5),
            "hr": np.stack([a[c][:n_hr].astype(np.int64) for c in HR_COLS], 1).reshape(n_hr, 6)}


def merge_tally_parts(parts: List[Dict[str, np.ndarray]]) -> Dict[str, np.ndarray]:
    """The union of the partitions' rows in first-batch-index order (the
    order of the unpartitioned hd_tally outputs)."""
    out = {}
    for key, rep_col in (("counts", 3), ("hr", 5)):
        rows = np.concatenate([p[key] for p in parts]) if parts else np.zeros((0, 5 if key == "counts" else 6),
                                                                               np.int64)
        out[key] = rows[np.argsort(rows[:, rep_col], kind="stable")]
    return out


def gather_tally(local: Dict[str, np.ndarray], world: int, device=None, group=None) -> Dict[str, np.ndarray]:
    """All-gather every rank's packed tally partition (sizes first, then the
    rows padded to the largest) and merge them.  device: where the
    collective runs (a CUDA device for RCCL, None = CPU for gloo)."""
    import torch
    import torch.distributed as dist
    if dist.get_backend(group) == "gloo":
        device = None
    sizes = torch.tensor([local["counts"].shape[0], local["hr"].shape[0]], dtype=torch.int64, device=device)
    all_sizes = torch.empty(2 * world, dtype=torch.int64, device=device)
    dist.all_gather_into_tensor(all_sizes, sizes, group=group)
    all_sizes = all_sizes.view(world, 2).cpu().numpy()
    parts = [dict() for _ in range(world)]
    for j, (key, cols) in enumerate((("counts", 5), ("hr", 6))):
        width = max(1, int(all_sizes[:, j].max()))
        pad = np.zeros((width, cols), np.int64)
        pad[: local[key].shape[0]] = local[key]
        out = torch.empty(world * width * cols, dtype=torch.int64, device=device)
        dist.all_gather_into_tensor(out, torch.from_numpy(pad.ravel()).to(device), group=group)
        got = out.view(world, width, cols).cpu().numpy()
        for r in range(world):
            parts[r][key] = got[r, : int(all_sizes[r, j])]
    return merge_tally_parts(parts)
