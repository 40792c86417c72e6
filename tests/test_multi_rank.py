"""Multi-rank sharding on CPU: world_size 2 (and 3) gloo process groups run the
shard/all-gather logic of the multi-GPU path on oracle-verified bitmaps and
reproduce the single-rank bitmap and tally exactly."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from hyperdrive_amd.shard import gather_bitmaps, shard_range


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
