#!/usr/bin/env python3
"""Benchmark: verified consensus msgs/s (secp256k1) on MI355X.

Workload (BASELINE.json configs[1]): batch-verify 1,048,576 synthetic
Prevote/Precommit messages from 100 signatories per GPU (SURVEY §8(d) C2:
signer = i % 100, type = 2 + (i/100)%2, h = 1 + i/200, r = 0; 90 % canonical
value, 5 % nil, 5 % random), seeded, signed with RFC6979 on the GPU before the
timed region.  One step = the hot path over one batch: verification (digest
-> recover / known-key check -> signatory -> Equal(From) -> admitted; verdict,
recovered signatory and valid bitmap written for every message) of this
rank's shard and the first-wins 2f+1 tally of it (N > 1: with the exchange
below).  Inputs are resident in HBM when timing starts.

Multi-GPU: one process per GPU, weak scaling: rank k generates and verifies
only messages [k*B, (k+1)*B) of the N*B-message stream (C4 generator;
--global-batch: one C4 batch split over the ranks).  `bench.py --gpus N`
under torch.distributed.run uses the launcher's ranks; without a launcher
(no WORLD_SIZE) it starts the N ranks itself as child processes
(launch_ranks) and relays rank 0's line.  Each rank tallies its own shard;
per step the ranks all-gather only their lexicographic (height, round)
ranges, and only the candidates of rounds inside another rank's range (the
rounds a shard boundary cuts) are routed to the round's owner over RCCL; each
rank keeps the rows it tallied, and the rows of all ranks are merged once,
after the timed region, for the line's totals (hyperdrive_amd/shard.py).  The
line reports ranks_seen (the process group's size) and, per rank, its device,
shard, timed span and routed_out / routed_in.

Defaults: 400 timed steps after 10 warm-up steps (about 0.6 s timed).  The
timed region includes the three-stream pipeline's fill and its drain (the
last step's tally); over 20 steps that fixed ~2.4 ms is 7 % of the region
(DESIGN.md §5, round 6).

Prints ONE JSON line on rank 0, with:
  roofline      the dominant kernel (k_fast_sums) timed live with HIP events
                on the library's stream (hd_ctx_profile), its algorithmic
                int32 work per message, and the verify call as a whole;
  cpu_baseline  the C restatement of the same path (oracle/hd_oracle.c) on the
                host's cores over a bounded sample, with a bit-exact check
                against the GPU's outputs for the same messages;
  sub           BASELINE configs C3 (1000 signatories, 64 rounds) and C5
                (30 % adversarial) on one GPU, and the cold first batch.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

W_OPS_PER_MSG = 6.06e5          # algorithmic int32 ops per Prevote/Precommit (full recovery)
# The same cost model (M = one 256-bit modular multiply = 160 int32 ops) for
# the known-key check R == s^-1 (m G + r P) that VALID messages of known
# signatories take, for the geometry the context reports
# (hd_ctx_fastpath_geometry): one table point per window, the first loaded and
# the rest mixed additions in XYZZ coordinates (8M + 2S = 10 M each, round 4;
# 8M + 3S = 11 M in Jacobian before); s^-1 mod n (296 M, as SURVEY's r^-1) and
# the inverse of ZZ ZZZ mod p (274 M) once per `per_inv` messages; Montgomery's
# trick (3 M per message and kind), u1 and u2 (2 M), the affine form (3 M) and
# comparison (2 M); one SHA-256 compression (2,200 ops).
M_OPS = 160
M_PER_ADD = 10                  # an XYZZ mixed addition, 8M + 2S (hd_fixedbase.h gxz_add_ge_nx)


def fast_ops_per_msg(g_windows, key_windows, per_inv):
    adds = g_windows + key_windows - 1
    return (adds * M_PER_ADD + (296 + 274) / per_inv + 2 * 3 + 2 + 5) * M_OPS + 2200


def sums_ops_per_msg(g_windows, key_windows):
    """k_fast_sums alone: the mixed additions, 10 M each, its prologue's
    u1 = m / s and u2 = r / s, 2 M, and the stored form (X ZZZ, Y ZZ, ZZ ZZZ),
    3 M."""
    return ((g_windows + key_windows - 1) * M_PER_ADD + 2 + 3) * M_OPS


BYTES_PER_MSG = 146 + 33        # HBM in + out per message
# INT32 VALU peak of one MI355X: 256 CU x 4 SIMD x 32 lanes x 2.4 GHz (the
# FP32-vector issue rate of MI355X_MICROARCH.md, 157.3 TFLOPS / 2 per FMA)
VALU_PEAK_OPS = 256 * 4 * 32 * 2.4e9


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=1 << 20, help="messages per GPU (weak scaling)")
    ap.add_argument("--global-batch", type=int, default=0,
                    help="messages over all GPUs (strong scaling; C4 = 16777216), split into contiguous shards")
    ap.add_argument("--signers", type=int, default=100)
    ap.add_argument("--adv", type=int, default=0, help="adversarial percentage (C5)")
    ap.add_argument("--cpu-sample", type=int, default=1 << 20,
                    help="messages of the CPU-baseline sample (~8 s on 16 host threads)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0: the host cores this process may use")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-tally", action="store_true")
    ap.add_argument("--stream-priority", choices=("high", "normal"), default="high",
                    help="priority of the verify stream")
    ap.add_argument("--tally-priority", choices=("high", "normal"), default="normal",
                    help="priority of the tally stream")
    ap.add_argument("--no-aux", action="store_true", help="skip the SURVEY §8(f) side measurements")
    ap.add_argument("--no-sub", action="store_true", help="skip the C3 / C5 sub-benchmarks")
    ap.add_argument("--sub-steps", type=int, default=100)
    ap.add_argument("--no-c4-check", action="store_true",
                    help="skip the untimed full-size bit-exact check of a 16M 30 %% adversarial C4 batch")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL, one GPU per rank) or gloo: a rehearsal of the N > 1 path with ranks "
                         "sharing the visible GPUs and host-side collectives")
    return ap.parse_args(argv)


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_env(base, rank: int, world: int, port: int) -> dict:
    """The environment torch.distributed.run gives rank `rank` of a one-node
    job of `world` ranks (env:// rendezvous on 127.0.0.1)."""
    env = dict(base)
    env.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                "LOCAL_WORLD_SIZE": str(world), "GROUP_RANK": "0", "MASTER_ADDR": "127.0.0.1",
                "MASTER_PORT": str(port)})
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")     # RCCL's dmabuf IPC on this pool
    return env


def launch_ranks(args, argv, child=None, device_count=None, timeout=None) -> int:
    """`bench.py --gpus N` without an external launcher: start N child
    processes, one per rank (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set as
    torch.distributed.run sets them), relay rank 0's JSON line and return the
    exit status.  This process never touches the GPU (torch.cuda.device_count()
    does not initialise it on this image) and never execs: the ranks are
    children.  With nccl (RCCL, one GPU per rank) more ranks than visible GPUs
    is refused before any rank starts.  The line is dropped (status 1) unless
    rank 0 reports ranks_seen == n_gpus == N."""
    import subprocess
    n = args.gpus
    if args.dist_backend == "nccl":
        if device_count is None:
            import torch
            device_count = torch.cuda.device_count()
        if n > device_count:
            print(json.dumps({"error": f"--gpus {n} with the nccl backend needs {n} GPUs, "
                                       f"torch.cuda.device_count() = {device_count}"}), flush=True)
            print(f"bench.py: --gpus {n} > {device_count} visible GPU(s); nccl (RCCL) needs one GPU per rank "
                  f"(use --dist-backend gloo to rehearse several ranks on fewer GPUs)", file=sys.stderr)
            return 2
    port = free_port()
    cmd = child or [sys.executable, "-u", os.path.abspath(__file__)]
    procs = []
    for r in range(n):
        procs.append(subprocess.Popen(cmd + list(argv), env=rank_env(os.environ, r, n, port),
                                      stdout=subprocess.PIPE if r == 0 else None, text=True))
    import threading
    lines = []

    def relay():
        for line in procs[0].stdout:                    # rank 0's stdout; progress stays visible
            line = line.rstrip("\n")
            if line.startswith("{"):
                lines.append(line)
            else:
                print(line, flush=True)

    reader = threading.Thread(target=relay, daemon=True)
    reader.start()
    t0 = time.monotonic()
    try:
        # poll every rank: one that fails ends the job (the others would wait
        # in a collective for it forever)
        while any(p.poll() is None for p in procs):
            if any(p.poll() not in (None, 0) for p in procs):
                break
            if timeout is not None and time.monotonic() - t0 > timeout:
                print(f"bench.py: ranks still running after {timeout} s", file=sys.stderr)
                break
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
        rcs = [p.wait() for p in procs]
        reader.join(timeout=10)
    bad = [(r, rc) for r, rc in enumerate(rcs) if rc != 0]
    if bad:
        for line in lines:
            print(line, flush=True)
        print(f"bench.py: rank(s) failed: {bad}", file=sys.stderr)
        return 1
    if not lines:
        print("bench.py: rank 0 printed no result line", file=sys.stderr)
        return 1
    try:
        out = json.loads(lines[-1])
    except ValueError:
        print(f"bench.py: rank 0's result line is not JSON: {lines[-1][:200]}", file=sys.stderr)
        return 1
    if out.get("ranks_seen") != n or out.get("n_gpus") != n:
        print(json.dumps({"error": f"launched {n} ranks but rank 0 saw ranks_seen={out.get('ranks_seen')}, "
                                   f"n_gpus={out.get('n_gpus')}"}), flush=True)
        return 1
    print(lines[-1], flush=True)
    return 0


def cpu_baseline(args, S):
    """The C restatement of the reference path (test infrastructure: the
    baseline leg only)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import subprocess
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    from oracle_c import COracle
    return COracle(os.path.join(ROOT, "oracle", "_build", "liboracle.so"))


def glv_port():
    """The 'port-glv' CPU baseline (oracle/glv_port.cpp; the baseline leg only)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import subprocess
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    from oracle_c import GlvPort
    return GlvPort(os.path.join(ROOT, "oracle", "_build", "libglvport.so"))


def secp_port():
    """The 'port-secp-class' CPU baseline (oracle/secp_port.cpp; the baseline leg only)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import subprocess
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    from oracle_c import SecpPort
    return SecpPort(os.path.join(ROOT, "oracle", "_build", "libsecpport.so"))


def _extra_streams(dev, priority, k):
    """The extra verify streams, created once per device and shared by every
    Pipeline of the process: the runtime maps streams onto the device's few
    hardware queues (GPU_MAX_HW_QUEUES, 4) round robin, so streams created per
    Pipeline would end up sharing a queue with the headline's or the tally's
    and serialise behind its kernels."""
    from hyperdrive_amd.device import verify_streams
    return verify_streams(dev, k + 1, priority)[1:]


class Pipeline:
    """verify (library streams `ws`, alternating) -> tally (stream `ts`) for
    one batch shape, with NBUF output buffers: the tally of step k runs on its
    own stream while the verifications of steps k+1 .. k+NBUF-1 are queued,
    so the tally's host syncs never drain the verify queue; consecutive
    verifications go to different streams, so the device runs step k+1's
    kernels in the SIMD slots step k's inversion kernels, last k_fast_sums
    round and fallback recovery leave idle (the library's per-call scratch
    sets, hd_fastverify.hip FbWork); every step's verification and tally
    complete inside the timed region.

    N > 1 (one process per GPU): `db` is this rank's shard only (global
    indices lo .. lo + B - 1).  The tally: the rank tallies its shard
    (hd_tally_device_bitmap, reps + lo); the ranks all-gather their round sets
    (shard.shared_rounds); the candidates of rounds present in more than one
    shard go to the owners of those rounds over RCCL
    (shard.route_candidates(rounds=...) / exchange_routed: one all-to-all of
    the counts, one of the 64-byte rows), each owner tallies what it received
    (hd_tally_routed_device); every rank keeps its local rows of the other
    rounds (shard.drop_rounds) and the small tables are all-gathered and
    merged (gather_tally_device)."""
    NBUF = int(os.environ.get("HD_BENCH_NBUF", 4))
    VSTREAMS = int(os.environ.get("HD_BENCH_VSTREAMS", 3))

    def __init__(self, v, db, total, lo, rank, world, dist, ws, ts, tally=True):
        import torch
        self.v, self.db, self.total, self.B, self.lo = v, db, total, db.n, lo
        self.rank, self.world, self.dist, self.ws, self.ts = rank, world, dist, ws, ts
        self.do_tally = tally
        dev = db.height.device
        self.dev = dev
        B = db.n
        assert B % 32 == 0
        self.wss = [ws] + _extra_streams(dev, ws.priority, self.VSTREAMS - 1)
        self.shard = db.c_struct()
        self.verdicts = [torch.empty(B, dtype=torch.uint8, device=dev) for _ in range(self.NBUF)]
        self.recovered = [torch.empty((B, 32), dtype=torch.uint8, device=dev) for _ in range(self.NBUF)]
        self.bitmaps = [torch.zeros(B // 32, dtype=torch.int32, device=dev) for _ in range(self.NBUF)]
        self.t_out, self.t_arr = v._tally_struct(B, pinned=True)
        if os.environ.get("HD_BENCH_NO_DUP"):      # A/B probe: skip the per-message classification download
            self.t_out.dup = None
        self.t_part = None
        self.route_rows = None
        if dist is not None:
            from hyperdrive_amd.shard import tally_out
            # the shard's own tally, and the owner's tally of the shared rounds
            # it received (separate pinned outputs: the first one's uploads may
            # still be reading its stage); sized for a skewed batch
            self.t_part = tally_out(v, B, pinned=True)
            self.t_own = tally_out(v, total, pinned=True)
        self.tally_info = {}
        self.tally_s = []            # host wall time of each synchronous tally (its thread)
        self.phase_s = {}            # N > 1: host time per phase of the exchange, summed
        self.last_tally = None
        # HD_BENCH_ASYNC_TALLY=1 (single GPU): the tally is queued without a
        # host wait (hd_tally_device_bitmap_async) and a collector thread
        # unpacks it.  Off by default: measured +3-5 % on C3 but the headline
        # C2 pipeline stalled for ~6 ms every few steps inside the submit
        # (DESIGN.md §4), so the tally thread with the synchronous call stays.
        # (=2: the collector thread also submits, one tally ahead of the one it collects)
        self.async_tally = world == 1 and bool(os.environ.get("HD_BENCH_ASYNC_TALLY"))
        self.async_mode = int(os.environ.get("HD_BENCH_ASYNC_TALLY", "0") or 0)
        self.tickets = [None] * self.NBUF
        self.ticket_objs = [None] * self.NBUF   # hd_tally_ticket per slot (its event is reused)
        self.stages = [None] * self.NBUF
        self.tally_retries = 0
        import threading
        self.tally_lock = threading.Lock()   # submit (this thread) and collect (the collector) share tally state
        self.tally_group = None   # set by main() for RCCL ranks
        self.range_group = None   # HD_BENCH_RANGE_GLOO: a gloo group for the per-step range exchange
        self.host_trace = [] if os.environ.get("HD_BENCH_HOSTTRACE") else None

    def verify(self, k):
        import torch
        buf = k % self.NBUF
        ws = self.wss[k % len(self.wss)]
        self.v.verify_batch_device(self.shard, self.verdicts[buf].data_ptr(), self.recovered[buf].data_ptr(), None,
                                   self.bitmaps[buf].data_ptr(), ws.cuda_stream)
        done = torch.cuda.Event()
        done.record(ws)
        return self.bitmaps[buf], done

    def _stage(self, j, need):
        from hyperdrive_amd import _lib
        lib = _lib.load()
        cur = self.stages[j]
        if cur is not None and cur[1] >= need:
            return cur
        if cur is not None:
            lib.hd_host_free(cur[0])
        ptr = ctypes.c_void_p()
        cap = need + need // 2
        rc = lib.hd_host_alloc(cap, ctypes.byref(ptr))
        if rc != 0:
            raise _lib.HDError(rc, "hd_host_alloc", "")
        self.stages[j] = (ptr.value, cap)
        return self.stages[j]

    def tally_submit(self, k, pending):
        """Queue tally k on the tally stream (after verification k, a device
        wait) with its results downloaded into stage k % NBUF; no host wait."""
        from hyperdrive_amd import _lib
        bitmap, done = pending
        self.ts.wait_event(done)
        if self.host_trace is not None:
            self.host_trace.append(("w", k, time.perf_counter()))
        lib = _lib.load()
        j = k % self.NBUF
        dup = 1 if self.t_out.dup else 0
        if self.ticket_objs[j] is None:
            self.ticket_objs[j] = _lib.HdTallyTicket()
        t = self.ticket_objs[j]
        with self.tally_lock:
            rc = self._submit_locked(lib, j, dup, t, bitmap)
        if rc != 0:
            raise _lib.HDError(rc, "hd_tally_device_bitmap_async", lib.hd_ctx_last_error(self.v.handle).decode())
        self.tickets[j] = (t, bitmap)

    def _submit_locked(self, lib, j, dup, t, bitmap):
        from hyperdrive_amd import _lib
        rc = 0
        for _ in range(2):
            stage, cap = self._stage(j, lib.hd_tally_stage_bytes(self.v.handle, self.B, dup))
            t.stage, t.stage_cap, t.dup = stage, cap, dup
            rc = lib.hd_tally_device_bitmap_async(self.v.handle, ctypes.byref(self.shard), bitmap.data_ptr(),
                                                  ctypes.byref(t), self.ts.cuda_stream)
            if rc != _lib.HD_ECAP:
                break
        return rc

    def tally_collect(self, k):
        """Wait for tally k's download and unpack it (HD_EAGAIN: more groups
        than staged -- tally the same inputs synchronously)."""
        from hyperdrive_amd import _lib
        j = k % self.NBUF
        t, bitmap = self.tickets[j]
        lib = _lib.load()
        tr = self.host_trace
        if tr is not None:
            tr.append(("c0", k, time.perf_counter()))
        # the wait for the download happens inside the foreign call (no GIL)
        rc = lib.hd_tally_collect(self.v.handle, ctypes.byref(t), ctypes.byref(self.t_out))
        if tr is not None:
            tr.append(("c1", k, time.perf_counter()))
        with self.tally_lock:
            if rc == _lib.HD_EAGAIN:
                self.tally_retries += 1
                rc = lib.hd_tally_device_bitmap(self.v.handle, ctypes.byref(self.shard), bitmap.data_ptr(),
                                                ctypes.byref(self.t_out), self.ts.cuda_stream)
        if rc != 0:
            raise _lib.HDError(rc, "hd_tally_collect", lib.hd_ctx_last_error(self.v.handle).decode())
        self.tally_info = {"n_hr": self.t_out.n_hr, "n_counts": self.t_out.n_counts}
        self.last_tally = (self.t_out, self.t_arr)
        self.tickets[j] = None

    def tally(self, pending):
        if pending is None or not self.do_tally:
            return
        t0 = time.perf_counter()
        try:
            self._tally(pending)
        finally:
            self.tally_s.append(time.perf_counter() - t0)

    def _tally(self, pending):
        import numpy as np
        import torch
        from hyperdrive_amd import _lib
        bitmap, done = pending
        self.ts.wait_event(done)
        if self.dist is None:
            lib = _lib.load()
            rc = lib.hd_tally_device_bitmap(self.v.handle, ctypes.byref(self.shard), bitmap.data_ptr(),
                                            ctypes.byref(self.t_out), self.ts.cuda_stream)
            if rc != 0:
                raise _lib.HDError(rc, "hd_tally_device_bitmap", lib.hd_ctx_last_error(self.v.handle).decode())
            self.tally_info = {"n_hr": self.t_out.n_hr, "n_counts": self.t_out.n_counts}
            self.last_tally = (self.t_out, self.t_arr)
            return
        from hyperdrive_amd.shard import (drop_pairs_rows, exchange_ranges, exchange_routed, pack_tally,
                                          ranges_overlap, round_range, route_candidates, routed_round_mask,
                                          tally_routed_host, unroute)
        lib = _lib.load()
        s = self.ts.cuda_stream
        g = self.tally_group
        ph = self.phase_s
        tp = time.perf_counter
        with torch.cuda.stream(self.ts):
            t0 = tp()
            t, a = self.t_part
            rc = lib.hd_tally_device_bitmap_part(self.v.handle, ctypes.byref(self.shard), bitmap.data_ptr(), 0, 1,
                                                 ctypes.byref(t), s)
            if rc != 0:
                raise _lib.HDError(rc, "hd_tally_device_bitmap_part", lib.hd_ctx_last_error(self.v.handle).decode())
            nh = t.n_hr
            hh, hr_ = a["hr_height"][:nh], a["hr_round"][:nh]
            t1 = tp()
            # the one per-step collective when no round straddles a shard edge
            rg = self.range_group
            ranges = exchange_ranges(round_range(hh, hr_), self.world, group=rg or g,
                                     device=None if rg is not None else self.dev)
            t2 = tp()
            local = pack_tally(a, t.n_counts, nh)          # host rows of the shard
            local["counts"][:, 3] += self.lo                # reps -> global indices
            local["hr"][:, 5] += self.lo
            mine = local
            routed_out = routed_in = n_routed = 0
            if ranges_overlap(ranges):                      # (identical on every rank)
                m = routed_round_mask(hh, hr_, ranges, self.rank)
                rh, rr = hh[m].astype(np.int64), hr_[m].astype(np.int64)
                n_routed = int(m.sum())
                order = np.lexsort((rr, rh))
                rounds = torch.from_numpy(np.stack([rh[order], rr[order]], 1).reshape(-1, 2)).to(self.dev)
                rows, counts = route_candidates(self.v, self.shard, bitmap.data_ptr(), self.lo, self.world, s,
                                                rows=self.route_rows, rounds=rounds)
                self.route_rows = rows
                recv = exchange_routed(rows, counts, self.world, group=g)
                routed_out, routed_in = int(sum(counts)), int(recv.shape[0])
                mine = {"counts": drop_pairs_rows(local["counts"], rh, rr), "hr": local["hr"][~m]}
                if routed_in:
                    db, gidx = unroute(self.v, recv, s)
                    own = tally_routed_host(self.v, db, gidx, s, self.t_own)
                    mine = {k: np.concatenate([mine[k], own[k]]) for k in mine}
            t3 = tp()
        for k, dt in (("local", t1 - t0), ("ranges", t2 - t1), ("route", t3 - t2)):
            ph.setdefault(k, []).append(dt)
        self.tally_info = {"n_hr_this_rank": int(len(mine["hr"])), "n_counts_this_rank": int(len(mine["counts"])),
                           "routed_rounds": n_routed, "routed_in": routed_in, "routed_out": routed_out}
        self.last_tally = mine

    def run(self, steps):
        """steps verifications + tallies.  The tallies run on a host thread of
        their own (each waits, on the device, for its verification): a tally
        synchronises its stream several times, and from the verifying thread
        those waits would hold back the next verification's enqueue -- the
        verify streams must always have the next call queued, so that it
        starts in the idle SIMD slots of the previous one.  Buffer k % NBUF is
        rewritten by verify(k + NBUF), issued only after tally(k) returned.
        The library calls release the GIL; verification and tally touch
        disjoint state of the context."""
        if self.async_tally:
            # verification k and tally k are queued by this thread without a
            # host wait (hd_tally_device_bitmap_async); a collector thread waits
            # for each tally's download in order and unpacks it, which frees
            # buffer k % NBUF for verification k + NBUF
            import queue
            import threading
            tr = self.host_trace
            free = threading.Semaphore(self.NBUF)
            work = queue.Queue()
            errors = []

            def collector():
                while True:
                    k = work.get()
                    if k is None:
                        return
                    try:
                        if not errors:
                            self.tally_collect(k)
                    except Exception as e:          # re-raised by run()
                        errors.append(e)
                    finally:
                        free.release()

            def submit_collector():
                # mode 2: submit tally k, then collect tally k - 1
                prev = None
                while True:
                    item = work.get()
                    try:
                        if item is not None and not errors:
                            self.tally_submit(item[0], item[1])
                        if prev is not None and not errors:
                            self.tally_collect(prev)
                    except Exception as e:          # re-raised by run()
                        errors.append(e)
                    finally:
                        if prev is not None:
                            free.release()
                    if item is None:
                        return
                    prev = item[0]

            th = threading.Thread(target=submit_collector if self.async_mode == 2 else collector, daemon=True)
            th.start()
            try:
                for k in range(steps):
                    free.acquire()
                    if errors:
                        break
                    if tr is not None:
                        tr.append(("v", k, time.perf_counter()))
                    pending = self.verify(k)
                    if not self.do_tally:
                        free.release()
                    elif self.async_mode == 2:
                        work.put((k, pending))
                    else:
                        self.tally_submit(k, pending)
                        if tr is not None:
                            tr.append(("s", k, time.perf_counter()))
                        work.put(k)
            finally:
                work.put(None)
                th.join()
            if errors:
                raise errors[0]
            return
        import queue
        import threading
        tr = self.host_trace
        work = queue.Queue()
        free = threading.Semaphore(self.NBUF)
        errors = []

        def tallies():
            while True:
                item = work.get()
                if item is None:
                    return
                try:
                    if not errors:
                        if tr is not None:
                            tr.append(("t", item[0], time.perf_counter()))
                        self.tally(item[1])
                except Exception as e:          # re-raised by run()
                    errors.append(e)
                finally:
                    free.release()

        th = threading.Thread(target=tallies, daemon=True)
        th.start()
        try:
            for k in range(steps):
                free.acquire()
                if errors:
                    break
                if tr is not None:
                    tr.append(("v", k, time.perf_counter()))
                work.put((k, self.verify(k)))
        finally:
            work.put(None)
            th.join()
        if errors:
            raise errors[0]

    def last(self, steps):
        buf = (steps - 1) % self.NBUF
        return self.verdicts[buf], self.recovered[buf], self.bitmaps[buf]

    def close(self):
        """Release the asynchronous tally's tickets (their events) and pinned
        stages (include/hd_verify.h hd_tally_ticket_release, hd_host_free)."""
        from hyperdrive_amd import _lib
        lib = _lib.load()
        for j, t in enumerate(self.ticket_objs):
            if t is not None:
                lib.hd_tally_ticket_release(ctypes.byref(t))
                self.ticket_objs[j] = None
        for j, st in enumerate(self.stages):
            if st is not None:
                lib.hd_host_free(st[0])
                self.stages[j] = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def timed(pipe, steps, dist, dev):
    import torch
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t = time.perf_counter()
    pipe.run(steps)
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    return time.perf_counter() - t


def main():
    argv = sys.argv[1:]
    args = parse(argv)
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no external launcher: this process starts the ranks itself
        sys.exit(launch_ranks(args, argv))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(json.dumps({"error": f"WORLD_SIZE={world} but --gpus {args.gpus}"}), flush=True)
        sys.exit(1)
    import numpy as np
    import torch

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        if args.dist_backend == "gloo":
            local = local % torch.cuda.device_count()
            torch.cuda.set_device(local)
            dist.init_process_group("gloo")
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    elif os.environ.get("HD_BENCH_FORCE_DIST"):
        # probe: one rank through the multi-rank tally path (RCCL group of 1):
        # the host-side cost of the exchange's orchestration without xGMI
        import torch.distributed as dist
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{free_port()}", world_size=1, rank=0,
                                device_id=torch.device("cuda", 0))
    else:
        dist = None
        torch.cuda.set_device(0)
    dev = torch.device("cuda", local if world > 1 else 0)

    import hyperdrive_amd as hd
    from hyperdrive_amd.device import generate, work_stream

    S = args.signers
    from hyperdrive_amd.shard import shard_range
    total = args.global_batch or args.batch * world
    lo, hi = shard_range(total, rank, world)
    B = hi - lo
    if B % 32 or B == 0:
        raise SystemExit(f"shard of {B} messages: use a global batch that splits into whole bitmap words")
    t0 = time.perf_counter()
    v = hd.Verifier(dev.index)                  # builds the device's shared G table (5.4 GB, once per process)
    ctx_s = time.perf_counter() - t0
    # the library's stream (created before anything else uses work_stream)
    ws = work_stream(dev, priority=-1 if args.stream_priority == "high" else 0)
    sigs, foreign = v.gen_keys(S)
    v.set_signatories(sigs)
    t0 = time.perf_counter()
    # this rank's shard only (messages lo .. hi - 1 of the seeded stream),
    # generated on its GPU: no rank holds another's messages
    db, _, _ = generate(v, 0, B, S, args.adv, keys=(sigs, foreign), start=lo, device=str(dev))
    gen_s = time.perf_counter() - t0

    torch.cuda.set_stream(ws)          # torch ops (RCCL all-gather included) share the library's stream
    ts = torch.cuda.Stream(device=dev, priority=-1 if args.tally_priority == "high" else 0)
    if os.environ.get("HD_BENCH_DEDICATED_TS"):
        # the tally stream on a hardware queue of its own (hd_stream_create_dedicated)
        from hyperdrive_amd import _lib
        sp = ctypes.c_void_p()
        if _lib.load().hd_stream_create_dedicated(v.handle, ctypes.byref(sp)) == 0:
            ts = torch.cuda.ExternalStream(sp.value, device=dev)
    pipe = Pipeline(v, db, total, lo, rank, world, dist, ws, ts, tally=not args.no_tally)
    if dist is not None and args.dist_backend == "nccl":
        pipe.tally_group = dist.new_group(backend="nccl")
        if os.environ.get("HD_BENCH_RANGE_GLOO"):    # A/B: the per-step range exchange over gloo (host)
            pipe.range_group = dist.new_group(backend="gloo")

    # The first batch on a fresh context is the cold start: every message
    # takes the full recovery, the first VALID message of each signatory
    # teaches the context its key and the per-key fixed-base tables are built
    # (stream-ordered, inside the call).  A long-lived replica has them from
    # earlier batches, so this pass is reported (cold_*), not timed.  Every
    # timed step still verifies every message.
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    pipe.run(1)
    torch.cuda.synchronize(dev)
    cold_s = time.perf_counter() - t0
    pipe.run(args.warmup)
    if pipe.host_trace is not None:
        pipe.host_trace.clear()
    elapsed = timed(pipe, args.steps, dist, dev)
    timed_tally_ms = [x * 1e3 for x in pipe.tally_s[-args.steps:]] or [0.0]
    if pipe.host_trace:
        t0h = pipe.host_trace[0][2]
        print("host trace:", [(a, k, round((t - t0h) * 1e3, 3)) for a, k, t in pipe.host_trace], file=sys.stderr)
    # Roofline pass (untimed for `value`): the same steps with one verify
    # stream, so that every k_fast_sums launch and verify call runs alone and
    # its HIP-event duration is its own (in the timed region consecutive calls
    # overlap and share the CUs)
    all_streams = pipe.wss
    pipe.wss = pipe.wss[:1]
    torch.cuda.synchronize(dev)
    v.profile(True)
    v.profile_read()                    # clear
    prof_s = timed(pipe, args.steps, dist, dev)
    calls, verify_ms, sums_launches, sums_ms = v.profile_read()
    v.profile(False)
    pipe.wss = all_streams
    own_elapsed = elapsed
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    verdict, recovered, bitmap = pipe.last(args.steps)
    known, fallback = v.fastpath_stats()
    ranks_seen, per_rank = 1, None
    if dist is not None:
        # what every rank saw: its device, shard, own timed span and tally exchange
        ranks_seen = dist.get_world_size()
        ts_ms = timed_tally_ms
        mine = {"rank": rank, "device": dev.index, "pid": os.getpid(), "shard": [lo, hi],
                "ms_per_step": own_elapsed / args.steps * 1e3,
                "tally_ms_mean": sum(ts_ms) / len(ts_ms), "tally_ms_max": max(ts_ms),
                "tally_phase_ms_median": {k: float(np.median(v[-args.steps:])) * 1e3 for k, v in pipe.phase_s.items()},
                "valid": int((verdict == 0).sum()), **pipe.tally_info}
        per_rank = [None] * ranks_seen
        dist.all_gather_object(per_rank, mine)
        # untimed: the ranks' rows (disjoint rounds) merged once, for the totals
        from hyperdrive_amd.shard import gather_tally_device
        last = pipe.last_tally
        merged = gather_tally_device({k: torch.from_numpy(np.ascontiguousarray(x)).to(dev) for k, x in last.items()},
                                     world)
        pipe.tally_info = {**pipe.tally_info, "n_hr": int(merged["hr"].shape[0]),
                           "n_counts": int(merged["counts"].shape[0]),
                           "note": "each rank keeps the rows of the rounds it tallied; n_hr / n_counts: all ranks' "
                                   "rows merged once after the timed region"}

    # correctness gate: without --adv every message of the workload is an honest
    # vote by construction, so every verdict must be VALID, every recovered
    # signatory its From and the valid bitmap full; a wrong kernel must not
    # produce a throughput number.
    hist = torch.bincount(verdict.long(), minlength=8).cpu().tolist()
    if args.adv == 0:
        full_bits = int(bitmap.view(torch.uint8).cpu().numpy().astype("uint8").sum())
        same_from = bool((recovered == db.frm).all())
        if hist[0] != B or full_bits != 255 * (B // 8) or not same_from:
            print(json.dumps({"error": "verification produced wrong outputs", "verdicts": hist}), flush=True)
            sys.exit(1)

    if rank == 0:
        ms_step = elapsed / args.steps * 1e3
        value = total * args.steps / elapsed
        geom = v.fastpath_geometry()
        w_fast = fast_ops_per_msg(*geom)
        w_sums = sums_ops_per_msg(geom[0], geom[1])
        live = B - fallback                      # messages of a step through the known-key check
        sums_avg = sums_ms / max(sums_launches, 1)
        call_avg = verify_ms / max(calls, 1)
        w_call = (live * w_fast + fallback * W_OPS_PER_MSG) / B
        achieved = live * w_sums / (sums_avg * 1e-3)
        out = {
            "metric": "verified consensus msgs/sec (secp256k1) at 1/2/4/8 MI355X; % INT32 VALU peak",
            "value": value,
            "unit": "msgs/s",
            "n_gpus": world,
            "ranks_seen": ranks_seen,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "strong" if args.global_batch else "weak",
            "vs_baseline": None,
            "dtype": "u32 (256-bit modular integer arithmetic)",
            "data": "synthetic (seeded RFC6979-signed votes generated on the GPU)",
            "config": {"workload": (f"C4: {total}-message batch sharded over {world} GPU(s) + 2f+1 tally"
                                    if args.global_batch else
                                    "C2: batch-verify 1M Prevote/Precommit from 100 signatories + 2f+1 tally"),
                       "messages_per_gpu": B, "global_batch": total, "signatories": S, "adversarial_pct": args.adv,
                       "outputs_per_step": "verdict, recovered signatory, valid bitmap, tally",
                       "parallelism": (f"shard-by-index x{world} (each rank holds, verifies and tallies only its "
                                       f"shard); round sets all-gathered, only rounds held by several ranks routed "
                                       f"to their owner (all-to-all); count rows all-gathered; backend "
                                       f"{'RCCL' if args.dist_backend == 'nccl' else args.dist_backend}"
                                       if world > 1 else "one GPU")},
            "roofline": {
                "bound": "valu",
                "kernel": "k_fast_sums (the known-key check's mixed additions; dominant kernel of the verify call)",
                "achieved": achieved / 1e12,
                "peak": VALU_PEAK_OPS / 1e12,
                "unit": "TOP/s (int32 lane-ops)",
                "frac": achieved / VALU_PEAK_OPS,
                "traffic": (pmc_traffic() or {}).get("sums_bytes_per_launch_corrected"),
                "kernel_ms": sums_avg,
                "launches_timed": sums_launches,
                "algorithmic_ops_per_msg": w_sums,
                "ops_model": "((g_windows + key_windows - 1) XYZZ mixed additions x 10 M + u1, u2 2 M + the stored form 3 M) x 160 int32 ops "
                             "(SURVEY §8(d) M); messages per launch = batch - fallback",
                "verify_call": {
                    "ms": call_avg,
                    "ops_per_msg": w_call,
                    "frac": B * w_call / (call_avg * 1e-3) / VALU_PEAK_OPS,
                    "frac_s8d": B * W_OPS_PER_MSG / (call_avg * 1e-3) / VALU_PEAK_OPS,
                    "frac_s8d_note": "SURVEY §8(d) prices the full recovery (W = 6.06e5 ops/msg, 3,761 M); the "
                                     "known-key check verifies the same identity with "
                                     f"{geom[0] + geom[1] - 1} fixed-base additions and shared inversions "
                                     f"({w_fast:.3g} ops/msg), so W/time exceeds the peak: it is "
                                     "recovery-equivalent throughput, not executed work",
                    "hbm_algorithmic_GBs": B * BYTES_PER_MSG / (call_avg * 1e-3) / 1e9,
                    "traffic": pmc_traffic(),
                },
                "geometry": {"g_windows": geom[0], "key_windows": geom[1], "msgs_per_inversion": geom[2]},
                "fallback_msgs_last_step": fallback, "known_signatories": known,
            },
            "verdicts": hist,
            "tally": pipe.tally_info,
            "tally_thread_ms": {"mean": sum(timed_tally_ms) / len(timed_tally_ms), "max": max(timed_tally_ms),
                                "note": "host wall time of each step's tally on its thread, from its start (queued behind its "
                                        "verification, whose end it waits for) to its results on the host (beside the next "
                                        "verifications), timed region only"},
            "cold": {"first_batch_s": cold_s, "cold_msgs_per_s": total / cold_s,
                     "ctx_create_s": ctx_s, "cold_msgs_per_s_incl_ctx": total / (cold_s + ctx_s),
                     "note": "first batch on a fresh context: full recovery of every message, key learning and "
                             "the per-key table build; ctx_create_s builds the shared G table"},
            "gen_s": gen_s,
            "one_stream_msgs_per_s": total * args.steps / prof_s,
            "verify_streams": len(all_streams),
            "tally_mode": "async" if pipe.async_tally else "thread", "tally_retries": pipe.tally_retries,
        }
        if per_rank is not None:
            out["dist_backend"] = args.dist_backend
            out["per_rank"] = per_rank
            out["distinct_devices"] = len({p["device"] for p in per_rank})
        if world == 1:
            out["oracle_sample_check"] = oracle_sample_check(db, verdict, recovered, sigs)
            if not args.no_aux:
                try:
                    out["aux"] = aux_benchmarks(v, db, ws)
                except Exception as e:  # reported, never fatal for the headline number
                    out["aux"] = {"error": repr(e)}
            if not args.no_cpu:
                try:
                    out["cpu_baseline"] = run_cpu_baseline(args, v, db, sigs, verdict, recovered)
                except Exception as e:  # reported, never fatal for the GPU number
                    out["cpu_baseline"] = {"error": repr(e)}
            if not args.no_sub:
                try:
                    out["sub"] = sub_benchmarks(args, v, sigs, foreign, dev, ws, ts)
                except Exception as e:
                    out["sub"] = {"error": repr(e)}
            if not args.no_c4_check:
                try:
                    out["c4_16m_bit_exact"] = c4_bit_exact(v, sigs, foreign, dev, ws)
                except Exception as e:  # reported, never fatal for the GPU number
                    out["c4_16m_bit_exact"] = {"error": repr(e)}
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def c4_bit_exact(v, sigs, foreign, dev, ws, n=1 << 24, adv=30):
    """Untimed: BASELINE configs[3] at full size with the C5 mix -- 16,777,216
    messages of the C4 generator (the headline's 100 signatories), 30 %
    adversarial across the 13 classes, verified by the headline's context
    (the product path, one call) and tallied by the library; then every
    verdict, recovered signatory, tally row and round decision is recomputed
    on the host (tests/bitexact.py: oracle/secp_port.cpp for the verdicts,
    oracle_tally for the rows and predicate bits; the checker, not the thing
    measured)."""
    import torch
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import bitexact
    from hyperdrive_amd.device import generate
    db, _, _ = generate(v, 0, n, len(sigs), adv, keys=(sigs, foreign), start=1 << 30, device=str(dev))
    verdict = torch.empty(n, dtype=torch.uint8, device=dev)
    rec = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    v.verify_batch_device(db.c_struct(), verdict.data_ptr(), rec.data_ptr(), None, None, ws.cuda_stream)
    ws.synchronize()
    gpu_s = time.perf_counter() - t0
    hb = db.to_host()
    del db
    res = bitexact.full_check(v, hb, verdict.cpu().numpy(), rec.cpu().numpy(), sigs)
    res.update({"adversarial_pct": adv, "gpu_verify_s": gpu_s, "stream_start": 1 << 30,
                "all_bit_exact": bool(res["verdicts"] and res["signatories"] and res["tally_rows"]
                                      and res["decisions"])})
    return res


def oracle_sample_check(db, verdict, recovered, sigs, n=512):
    """Untimed: 512 seeded messages of the last timed step against the C
    oracle (verdict and recovered signatory, bit for bit)."""
    import numpy as np
    import torch
    co = cpu_baseline(None, None)
    rng = np.random.default_rng(512)
    pick = np.sort(rng.choice(verdict.numel(), min(n, verdict.numel()), replace=False))
    p = torch.from_numpy(pick).to(db.height.device)
    from hyperdrive_amd.verify import Batch
    sb = Batch(db.type[p].cpu().numpy(), db.height[p].cpu().numpy(), db.round[p].cpu().numpy(),
               db.valid_round[p].cpu().numpy(), db.value[p].cpu().numpy(), db.frm[p].cpu().numpy(),
               db.sig[p].cpu().numpy())
    cv, crec = co.verify(sb, sigs, True, threads=8)
    ok_v = cv.tolist() == verdict[p].cpu().numpy().tolist()
    ok_r = crec.tobytes() == recovered[p].cpu().numpy().tobytes()
    return {"messages": len(pick), "verdicts_equal": ok_v, "recovered_equal": ok_r}


def sub_benchmarks(args, v, sigs, foreign, dev, ws, ts):
    """BASELINE configs beside the headline, on one GPU, steps of verify +
    tally after a key-learning pass: C5 (30 % adversarial, the headline's
    context and keys), a signatory-set change (100 -> 150 signatories on the
    same context) and C3 (1000 signatories, 64 rounds of 1 propose + 1000
    prevotes + 1000 precommits = 128,064 messages, a context of its own)."""
    import torch
    import hyperdrive_amd as hd
    from hyperdrive_amd.device import generate
    out = {}
    # C5: the C2 stream with 30 % of the messages corrupted across the classes
    B = args.batch
    db5, _, _ = generate(v, 0, B, args.signers, 30, keys=(sigs, foreign), device=str(dev))
    p5 = Pipeline(v, db5, B, 0, 0, 1, None, ws, ts)
    # untimed warm-up to the steady state: the first call recovers the foreign
    # senders' keys and claims their slots on the device; the host sees the
    # claims only once a call has completed, and the next call then builds
    # their tables (~20 ms). Without the syncs that build lands in the timed
    # steps (scripts/c5_probe.py: 3.33 ms per step on the first 20, then 2.14).
    for _ in range(3):
        p5.run(1)
        torch.cuda.synchronize(dev)
    p5.run(2)
    el = timed(p5, args.sub_steps, None, dev)
    vd, rec5, _ = p5.last(args.sub_steps)
    out["C5_adversarial_30pct"] = {"oracle_sample_check": oracle_sample_check(db5, vd, rec5, sigs),
                                   "messages": B, "msgs_per_s": B * args.sub_steps / el,
                                   "ms_per_step": el / args.sub_steps * 1e3,
                                   "verdicts": torch.bincount(vd.long(), minlength=8).cpu().tolist(),
                                   "fallback_msgs": v.fastpath_stats()[1], "tally": p5.tally_info}
    del p5, db5
    out["C5_ingress_out_of_order"] = ingress_c5(v, (sigs, foreign), args.signers, B, ws, str(dev))
    out["host_buffers_C2"] = host_buffers(v, args, sigs, foreign, dev)
    # Signatory-set change (ResetHeight with a new epoch's set): the C2
    # context switches to 150 signatories, the 100 it knows plus 50 new ones.
    # The first batch after the change learns the 50 keys and builds their
    # tables inside the verify call; later batches run at the steady rate.
    S6 = args.signers + 50
    k6 = v.gen_keys(S6)
    t0 = time.perf_counter()
    v.set_signatories(k6[0])
    set_s = time.perf_counter() - t0
    db6, _, _ = generate(v, 0, B, S6, 0, keys=k6, device=str(dev))
    p6 = Pipeline(v, db6, B, 0, 0, 1, None, ws, ts)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    p6.run(1)
    torch.cuda.synchronize(dev)
    first6 = time.perf_counter() - t0
    p6.run(2)
    el = timed(p6, args.sub_steps, None, dev)
    vd, _, _ = p6.last(args.sub_steps)
    out["set_change_100_to_150"] = {
        "messages": B, "set_signatories_s": set_s, "first_batch_s": first6, "first_batch_msgs_per_s": B / first6,
        "msgs_per_s": B * args.sub_steps / el, "ms_per_step": el / args.sub_steps * 1e3,
        "verdicts": torch.bincount(vd.long(), minlength=8).cpu().tolist(),
        "known_signatories": v.fastpath_stats()[0], "key_windows": v.fastpath_geometry()[1],
        "note": "hd_set_signatories keeps the known keys while the table width stays (the first batch learns the "
                "new ones: full recovery of their first messages, tables built in the same call); when 150 keys' "
                "tables no longer fit the width the 100 had, the context re-maps at the next width and the first "
                "batch learns every key again"}
    del p6, db6
    # C3: its own context (the 1000 keys' tables need the table budget the
    # C2 context holds: it is released first by the caller's order)
    S3 = 1000
    v3 = hd.Verifier(dev.index)
    k3 = v3.gen_keys(S3)
    v3.set_signatories(k3[0])
    n3 = 64 * (2 * S3 + 1)
    db3, _, _ = generate(v3, 1, n3, S3, 0, keys=k3, device=str(dev))
    n3p = (n3 + 31) // 32 * 32
    if n3p != n3:
        db3, _, _ = generate(v3, 1, n3p, S3, 0, keys=k3, device=str(dev))   # whole bitmap words
    p3 = Pipeline(v3, db3, n3p, 0, 0, 1, None, ws, ts)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    p3.run(1)
    torch.cuda.synchronize(dev)
    cold3 = time.perf_counter() - t0
    p3.run(8)
    # a C3 step is 0.28 ms: 8 x sub_steps of them (20M messages, as many as
    # the 1M-message lines time) keep host jitter out of the rate
    steps3 = 8 * args.sub_steps
    el = timed(p3, steps3, None, dev)
    vd, rec3, _ = p3.last(steps3)
    out["C3_1000_signatories_64_rounds"] = {
        "oracle_sample_check": oracle_sample_check(db3, vd, rec3, k3[0]),
        "messages": n3p, "steps": steps3, "msgs_per_s": n3p * steps3 / el, "ms_per_step": el / steps3 * 1e3,
        "verdicts": torch.bincount(vd.long(), minlength=8).cpu().tolist(), "fallback_msgs": v3.fastpath_stats()[1],
        "known_signatories": v3.fastpath_stats()[0], "key_windows": v3.fastpath_geometry()[1],
        "cold_first_batch_s": cold3, "tally": p3.tally_info}
    del p3, db3
    v3.close()
    out["many_signatories"] = many_signatories(args, dev, ws, ts)
    return out


def many_signatories(args, dev, ws, ts, sizes=(2000, 4000, 8000), steps=50):
    """The per-key table budget with thousands of signatories (replica.go:54,
    136-144: the admitted set and f): the C2 stream (1M messages, signer =
    i % S) from S = 2,000, 4,000 and 8,000 signatories, each on a context of
    its own (the headline's context keeps its tables beside it), with the
    default table width -- the widest whose tables for every key fit what is
    left of the device's budget: 16-bit windows (36 MB per key), then 13-bit
    (5 MB per key) -- and, at 8,000, with the 16-bit width forced (the
    round-5 tiers: the keys past the budget's slots get no table and take the
    full recovery, ~10x per message).  Per line: msgs/s over `steps` steps of
    verify + tally, keys with tables, the last step's full-recovery count."""
    import torch
    import hyperdrive_amd as hd
    from hyperdrive_amd.device import generate
    B = args.batch
    res = {}
    for S in sizes:
        for width in ((0, 16) if S == sizes[-1] else (0,)):
            vS = hd.Verifier(dev.index)
            try:
                if width:
                    vS.set_variant("key_width", width)
                ks = vS.gen_keys(S)
                vS.set_signatories(ks[0])
                db, _, _ = generate(vS, 0, B, S, 0, keys=ks, device=str(dev))
                p = Pipeline(vS, db, B, 0, 0, 1, None, ws, ts)
                torch.cuda.synchronize(dev)
                t0 = time.perf_counter()
                p.run(1)
                torch.cuda.synchronize(dev)
                cold = time.perf_counter() - t0
                for _ in range(2):              # tables of keys learned late are built by the next calls
                    p.run(1)
                    torch.cuda.synchronize(dev)
                el = timed(p, steps, None, dev)
                vd, rec, _ = p.last(steps)
                known, fallback = vS.fastpath_stats()
                res[f"S{S}_" + ("default" if not width else f"forced_{width}bit")] = {
                    "signatories": S, "messages": B, "msgs_per_s": B * steps / el, "ms_per_step": el / steps * 1e3,
                    "key_windows": vS.fastpath_geometry()[1], "keys_with_tables": known,
                    "full_recovery_msgs_last_step": fallback, "cold_first_batch_s": cold,
                    "all_valid_and_recovered": bool((vd == 0).all()) and bool((rec == db.frm).all())}
                p.close()
                del p, db
            finally:
                vS.close()
    res["note"] = ("C2 stream with S signatories; default: the context picks 22-, 20-, 16- or 13-bit key tables by "
                   "what is left of the device's table budget (64 GiB, the headline's context holding its "
                   "own); forced_16bit: every key past the budget's 16-bit slots takes the full recovery")
    return res


def host_buffers(v, args, sigs, foreign, dev, steps=12):
    """The cgo caller's path (replica.go:156-181 hands over host messages):
    the C2 batch in host memory through hd_verify_submit / hd_verify_wait,
    two tickets in flight, so batch k+1's upload runs under batch k's
    kernels.  PCIe-inclusive (inputs 146 B and outputs 33 B per message cross
    PCIe), hence never `value`.  Pinned buffers (hd_host_alloc-like, here torch
    pin_memory) move by DMA; pageable ones go through the library's staging."""
    import numpy as np
    import torch
    from hyperdrive_amd.device import generate
    from hyperdrive_amd.verify import Batch, CompactBatch
    B = args.batch
    INFLIGHT = 3    # tickets queued (the library keeps HD_HOST_SLOTS = 3 pipelines)
    db, _, _ = generate(v, 0, B, args.signers, 0, keys=(sigs, foreign), device=str(dev))
    hb = db.to_host()
    if np.isin(hb.type, (2, 3)).all():
        hb.valid_round = None   # votes only: a cgo caller passes no valid_round column (-1 = InvalidRound)
    keep = []

    def pinned(a):
        t = torch.empty(a.shape, dtype={np.uint8: torch.uint8, np.int64: torch.int64,
                                         np.uint16: torch.int16, np.uint32: torch.int32}[a.dtype.type], pin_memory=True)
        keep.append(t)
        o = t.numpy().view(a.dtype)
        o[...] = a
        return o

    res = {}
    cb = CompactBatch.from_batch(hb, sigs)
    for name, mk in (("pinned", pinned), ("pageable", lambda a: a.copy()), ("compact_pinned", pinned),
                     ("compact_pageable", lambda a: a.copy())):
        compact = name.startswith("compact")
        if compact:
            src = CompactBatch(*(mk(a) if a is not None else None for a in
                                 (cb.type, cb.height, cb.round, cb.valid_round, cb.from_idx, cb.value_idx, cb.sig,
                                  cb.escape, cb.values)))
            submit = v.submit_compact
            up = 86 * B + 32 * (len(cb.escape) + len(cb.values))
        else:
            src = Batch(*(mk(a) if a is not None else None for a in
                          (hb.type, hb.height, hb.round, hb.valid_round, hb.value, hb.frm, hb.sig)))
            submit = v.submit
            up = 146 * B
        outs = [(mk(np.zeros(B, np.uint8)), mk(np.zeros((B, 32), np.uint8)),
                 mk(np.zeros((B + 31) // 32, np.uint32))) for _ in range(INFLIGHT)]
        for k in range(INFLIGHT):                        # warm: staging and device buffers
            v.wait(submit(src, *outs[k % INFLIGHT]))
        t0 = time.perf_counter()
        pending = []
        for k in range(steps):
            pending.append(submit(src, *outs[k % INFLIGHT]))
            if len(pending) == INFLIGHT:              # at most INFLIGHT tickets queued
                v.wait(pending.pop(0))
        for t in pending:
            v.wait(t)
        dt = time.perf_counter() - t0
        ok = bool((outs[0][0] == 0).all() and (outs[0][1] == hb.frm).all())
        res[name] = {"msgs_per_s": B * steps / dt, "ms_per_batch": dt / steps * 1e3,
                     "h2d_bytes_per_batch": up, "h2d_GBs": up * steps / dt / 1e9, "outputs_ok": ok}
    res.update({"messages": B, "batches": steps, "in_flight": INFLIGHT, "compact_values": len(cb.values),
                "compact_escape_rows": len(cb.escape),
                "note": "PCIe-inclusive: 146 B up (compact form: 86 B, From and value as 16-bit indices, "
                        "hd_verify_submit_compact) and 33 B + bitmap down per message; bounded by the host link, "
                        "not by the kernels"})
    return res


def ingress_c5(v, keys, S, n, ws, dev, heights=64):
    """BASELINE config 5 through the replica ingress (hyperdrive_amd/ingress.py):
    the C2 stream with 30 % of the messages corrupted, shuffled so that heights
    arrive out of order, marshalled per message type to wire bytes.  A cycle:
    the push (unmarshal -> verify -> filterHeight -> mq insert with a
    per-sender capacity of 1000, every authenticated message buffered), then
    `heights` flushes with ResetHeight between (mq.Consume of the current
    height against procsAllowed -> vote logs).  Timed: 8 cycles back to back
    with cycle c+1's unmarshal + authentication on the device beside cycle c's
    flushes (replica.go:117-145, 251-264), and 3 serial cycles.  Checked:
    every cycle delivers exactly the VALID messages of heights 1..`heights`
    (the queues keep each sender's lowest heights, mq.go:125-142)."""
    import torch
    from hyperdrive_amd.codec import marshal_device
    from hyperdrive_amd.device import DeviceBatch, generate
    from hyperdrive_amd.ingress import Ingress
    db, _, _ = generate(v, 0, n, S, 30, keys=keys, device=dev)
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    perm = torch.randperm(n, device=dev, generator=g)
    parts = []
    for t in (2, 3):
        idx = perm[(db.type == t)[perm]]
        sub = DeviceBatch(int(idx.numel()), *(getattr(db, f)[idx].contiguous()
                                               for f in ("type", "height", "round", "valid_round", "value", "frm",
                                                         "sig")))
        parts.append((t, sub, marshal_device(v, t, sub, with_sig=True, stream=ws)))
    ing = Ingress(v, height=1, max_capacity=1000)
    for _ in range(2):   # warm: allocations on both streams, scratch sets of both buffer sizes, the
        ing.push_wires([(t, wire, sub.n) for t, sub, wire in parts])   # consume's mapped stage (first flush)
        ing.flush()
        ing.mq.drop_below(2 ** 62)
    wires = [(t, wire, sub.n) for t, sub, wire in parts]

    def restart():                  # the next cycle starts from height 1 and an empty queue
        ing.height = 1
        ing.votes.reset(1)
        ing._clean = None
        ing.mq.drop_below(2 ** 62)

    def flushes():
        got = 0
        for h in range(1, heights + 1):
            if h > 1:
                ing.reset_height(h)
            got += len(ing.flush().consumed)
        return got

    want = None
    # serial cycles (push, then the flushes), as in rounds 2-5; the median one
    reps = []
    for rep in range(3):
        restart()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        verdicts = ing.push_wires(wires)
        torch.cuda.synchronize()                      # push_ms includes the device work it queued
        t1 = time.perf_counter()
        delivered = flushes()
        t2 = time.perf_counter()
        reps.append((t2 - t0, t1 - t0, t2 - t1))
        if want is None:
            want = sum(int(((vd == 0) & (sub.height >= 1) & (sub.height <= heights)).sum())
                       for vd, (_, sub, _) in zip(verdicts, parts))
    tot, push, flush = sorted(reps)[1]
    serial_ok = delivered == want
    # overlapped cycles (the replica's steady state): cycle c+1's wire buffers
    # are unmarshalled and authenticated on the device (push_wires_begin)
    # while the host flushes cycle c's heights from the queue, and go into the
    # queue (push_finish: filterHeight + mq insert) after those flushes --
    # the reference's loop (replica.go:100-147) reaches a message only after
    # the ones before it.  Every cycle delivers exactly its VALID messages of
    # the flushed heights.
    C = 8
    restart()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    pend = ing.push_wires_begin(wires)
    per_cycle, flush_s, ok_all = [], 0.0, True
    for c in range(C):
        ing.push_finish(pend)                          # cycle c into the queue
        if c + 1 < C:
            pend = ing.push_wires_begin(wires)         # cycle c + 1 authenticating beside the flushes
        f0 = time.perf_counter()
        got = flushes()
        flush_s += time.perf_counter() - f0
        ok_all &= got == want
        per_cycle.append(got)
        if c + 1 < C:
            restart()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    vh = torch.bincount(torch.cat(verdicts).long(), minlength=9).cpu().tolist()
    buffered = len(ing.mq)
    ing.close()
    return {"messages": n, "total_msgs_per_s": n * C / el, "cycles": C, "ms_per_cycle": el / C * 1e3,
            "flush_ms_per_cycle": flush_s / C * 1e3, "flushes": heights,
            "delivered_per_cycle": per_cycle[0], "delivered_equals_valid_at_flushed_heights": bool(ok_all and serial_ok),
            "serial": {"push_ms": push * 1e3, "push_msgs_per_s": n / push, "flush_ms": flush * 1e3,
                       "total_msgs_per_s": n / tot, "reps_total_ms": [round(r[0] * 1e3, 3) for r in reps],
                       "reps_push_ms": [round(r[1] * 1e3, 3) for r in reps],
                       "reps_flush_ms": [round(r[2] * 1e3, 3) for r in reps],
                       "delivered": delivered, "delivered_equals_valid_at_flushed_heights": bool(serial_ok)},
            "verdicts": vh, "buffered_after": buffered,
            "note": "30 % adversarial C2 batch in random order (heights out of order), prevote and precommit wire "
                    "buffers; per cycle: authenticate -> filterHeight -> mq insert, then 64 flushes with "
                    "ResetHeight between (mq.Consume + vote logs).  total_msgs_per_s: 8 cycles back to back, each "
                    "cycle's unmarshal + authentication queued on the device while the host flushes the previous "
                    "cycle (Ingress.push_wires_begin / push_finish); serial: push then flushes, median of 3"}


HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: 8.0 TB/s spec (6.29 TB/s measured float4 copy)


def _time_ms(fn, ws, reps=5):
    """Average device time of fn() over reps launches on stream ws (HIP events)."""
    import torch
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(ws)
    for _ in range(reps):
        fn()
    e1.record(ws)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def aux_benchmarks(v, db, ws):
    """The SURVEY §8(f) rows around the hot path, measured on the same batch
    (not part of the headline value): the surge wire codec (HBM-bound), mq
    bulk insert, the digest lanes and the host vote table."""
    import ctypes
    import torch
    from hyperdrive_amd import _lib
    from hyperdrive_amd.codec import record_size
    from hyperdrive_amd.device import DeviceBatch
    lib = _lib.load()
    out = {}
    n = db.n
    S = record_size(2, True)
    buf = torch.empty(n * S, dtype=torch.uint8, device=db.height.device)
    cs = db.c_struct()
    dec = DeviceBatch.empty(n, str(db.height.device))
    co = dec.c_out()
    status = torch.empty(n, dtype=torch.uint8, device=db.height.device)

    def enc():
        rc = lib.hd_marshal_batch_device(v.handle, 2, 1, ctypes.byref(cs), buf.data_ptr(), buf.numel(), ws.cuda_stream)
        assert rc == 0, rc

    def decd():
        rc = lib.hd_unmarshal_batch_device(v.handle, 2, 1, buf.data_ptr(), buf.numel(), n, ctypes.byref(co),
                                           status.data_ptr(), ws.cuda_stream)
        assert rc == 0, rc

    ms_e = _time_ms(enc, ws)
    ms_d = _time_ms(decd, ws)
    ok = bool((dec.height == db.height).all()) and bool((dec.sig == db.sig).all()) and int(status.sum()) == 0
    # algorithmic bytes: record in + SoA out (type 1, h 8, r 8, value 32, from 32, sig 65, status 1)
    soa = 1 + 8 + 8 + 32 + 32 + 65
    for name, ms, byts in (("surge_unmarshal_signed_prevotes", ms_d, n * (S + soa + 1)),
                           ("surge_marshal_signed_prevotes", ms_e, n * (S + soa - 1))):
        gbs = byts / (ms * 1e-3) / 1e9
        out[name] = {"messages": n, "ms": ms, "msgs_per_s": n / (ms * 1e-3), "GBs": gbs,
                     "roofline": {"bound": "hbm", "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS},
                     "round_trip_ok": ok}
    # mq bulk insert (mq.go:103-143) of the verified batch: one queue per
    # From (the C2 signer i % S), per-sender capacity 1000 (opt.go:19), then a
    # full consume against the admitted set; wall time of the synchronous calls
    from hyperdrive_amd.mq import MessageQueue
    S = 100
    q = MessageQueue(v, 1000)
    q.insert_device(db, None, stream=ws)              # warm (allocations)
    q.consume(2 ** 62)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    q.insert_device(db, None, stream=ws)
    t1 = time.perf_counter()
    kept = len(q)
    b, _ = q.consume(2 ** 62)
    t2 = time.perf_counter()
    q.close()
    out["mq_bulk_insert"] = {"messages": n, "senders": S, "max_capacity": 1000, "kept": kept,
                             "insert_ms": (t1 - t0) * 1e3, "insert_msgs_per_s": n / (t1 - t0),
                             "consume_ms_incl_download": (t2 - t1) * 1e3, "consumed": len(b),
                             "ok": kept == S * 1000 and len(b) == kept}
    # digest lanes (include/hd_digest.h): preimage digests of the batch;
    # ~81 B of HBM per message (type, h, r, value in; 32 B out)
    from hyperdrive_amd.digest import KECCAK256, SHA256, digest_device
    dgo = torch.empty((n, 32), dtype=torch.uint8, device=db.height.device)
    for algo, name in ((SHA256, "sha256"), (KECCAK256, "keccak256")):
        ms = _time_ms(lambda: digest_device(v, algo, db, out=dgo, stream=ws), ws)
        out["digest_" + name] = {"messages": n, "ms": ms, "msgs_per_s": n / (ms * 1e-3),
                                 "GBs": n * 81 / (ms * 1e-3) / 1e9}
    # end-to-end replica ingress from wire bytes (hyperdrive_amd/ingress.py):
    # unmarshal -> verify -> filterHeight -> mq insert, then flush the
    # current height into the vote logs; wall time of the synchronous chain
    from hyperdrive_amd.codec import marshal_device
    from hyperdrive_amd.ingress import Ingress
    wire = marshal_device(v, 2, db, with_sig=True, stream=ws)
    ing = Ingress(v, height=1, max_capacity=1000)
    ing.push_wire(2, wire, n, stream=ws)                  # warm (allocations)
    ing.votes.reset(1)
    ing.mq.drop_below(2 ** 62)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    vg = ing.push_wire(2, wire, n, stream=ws)
    res = ing.flush()
    t1 = time.perf_counter()
    out["ingress_wire_to_votes"] = {"messages": n, "ms": (t1 - t0) * 1e3, "msgs_per_s": n / (t1 - t0),
                                    "valid": int((vg == 0).sum()), "consumed_height_1": len(res.consumed),
                                    "buffered": len(ing.mq)}
    ing.close()
    out["vote_table"] = vote_table_bench()
    return out


def vote_table_bench():
    """Host-side incremental vote logs (include/hd_votes.h) on the C3 shape:
    1000 signers x 64 rounds x (prevote + precommit) = 128,000 votes of one
    height inserted in arrival order, then every round's T-predicates
    (quorum.decide_votes: 6 O(1) lookups, through ctypes)."""
    import numpy as np
    from hyperdrive_amd.quorum import decide_votes, thresholds
    from hyperdrive_amd.verify import Batch
    from hyperdrive_amd.votes import INSERTED, VoteLog
    S, R = 1000, 64
    n = 2 * S * R
    i = np.arange(n)
    r = (i // (2 * S)).astype(np.int64)
    typ = (2 + i % 2).astype(np.uint8)
    frm = np.zeros((n, 32), np.uint8)
    frm[:, :4] = ((i // 2) % S).astype(np.uint32).view(np.uint8).reshape(n, 4)
    val = np.zeros((n, 32), np.uint8)
    val[:, 0] = 1
    val[:, 8:16] = r.view(np.uint8).reshape(n, 8)
    val[i % 20 == 7] = 0                                     # 5% nil
    b = Batch(typ, np.ones(n, np.int64), r, None, val, frm, np.zeros((n, 65), np.uint8))
    v = VoteLog(1)
    v.insert_batch(b)                                        # warm: tables grown once
    v.reset(1)
    t0 = time.perf_counter()
    st, _ = v.insert_batch(b)
    t1 = time.perf_counter()
    f = thresholds(S)[0]
    dec = [decide_votes(v, rr, f, val[2 * S * rr].tobytes(), True, rr - 1) for rr in range(R)]
    t2 = time.perf_counter()
    v.close()
    return {"votes": n, "insert_ms": (t1 - t0) * 1e3, "ns_per_vote": (t1 - t0) * 1e9 / n,
            "predicates_ms_64_rounds": (t2 - t1) * 1e3, "all_inserted": bool((st == INSERTED).all()),
            "commit_rounds": sum(d["commit"] for d in dec), "cores": 1}


def pmc_traffic():
    """HBM bytes per launch from the committed rocprofv3 PMC passes (separate
    FETCH_SIZE / WRITE_SIZE runs, KiB -> bytes, FETCH_SIZE doubled per
    MI355X_MICROARCH.md's gfx950 correction): k_fast_sums alone and the known-key
    check's kernels together, from the newest round under profiles/ that has
    them.  The table reads (24 x 64 B per message) dominate; the batch itself
    is 179 B/message."""
    rounds = sorted((d for d in os.listdir(os.path.join(ROOT, "profiles")) if d.startswith("round")),
                    key=lambda d: (int("".join(c for c in d[5:] if c.isdigit()) or 0), d), reverse=True)
    for rnd in rounds:
        base = os.path.join(ROOT, "profiles", rnd)
        try:
            with open(os.path.join(base, "pmc_k_fast_sums.json")) as fh:
                sums = json.load(fh)
            with open(os.path.join(base, "pmc_known_key_check.json")) as fh:
                call = json.load(fh)
        except (OSError, ValueError):
            continue
        try:
            return {"sums_bytes_per_launch_raw": sums["hbm_bytes_raw"],
                    "sums_bytes_per_launch_corrected": sums["hbm_bytes_corrected"],
                    "check_bytes_per_call_raw": call["hbm_bytes_raw"],
                    "check_bytes_per_call_corrected": call["hbm_bytes_corrected"],
                    "source": f"profiles/{rnd}/pmc_k_fast_sums.json, pmc_known_key_check.json "
                              "(rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE)"}
        except KeyError:
            continue
    return None


def cgroup_cpu_quota():
    """CPUs' worth of time the cgroup v2 quota grants (cpu.max), or None."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, period = fh.read().split()[:2]
        return None if q == "max" else max(1, int(int(q) / int(period)))
    except (OSError, ValueError):
        return None


def host_cpu_info():
    """(CPU model, cores this process may use, online CPUs of the host): the
    affinity mask bounded by the cgroup's CPU quota (a GPU box shows every
    CPU of the machine in its mask but grants one GPU's share of time; more
    threads than the quota only queue)."""
    model = ""
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        allowed = len(os.sched_getaffinity(0))
    except AttributeError:
        allowed = os.cpu_count() or 1
    quota = cgroup_cpu_quota()
    if quota:
        allowed = min(allowed, quota)
    return model, allowed, os.cpu_count() or allowed


def run_cpu_baseline(args, v, db, sigs, gpu_verdict, gpu_recovered):
    """The CPU path timed on the host's cores: the C
    restatement (oracle/hd_oracle.c, kind 'port') verifies the first
    --cpu-sample messages of the same workload (digest -> recover ->
    signatory -> Equal(From) -> admitted), then tallies them (first-wins logs
    and counts, oracle_tally) and evaluates the quorum predicates of every
    (height, round) with f = len(signatories) / 3 and the round's canonical
    value as the propose.  Timed on every host thread this process may use,
    and again on the per-GPU share (OMP_NUM_THREADS); the verdicts, recovered
    signatories, tally rows and decisions are checked bit for bit against the
    GPU's for the same messages (untimed)."""
    import numpy as np
    co = cpu_baseline(args, None)
    import hd_pyoracle as O
    from hyperdrive_amd import quorum
    n = min(args.cpu_sample, db.n, gpu_verdict.numel())
    host = db.to_host()
    from hyperdrive_amd.verify import Batch
    sample = Batch(host.type[:n].copy(), host.height[:n].copy(), host.round[:n].copy(), host.valid_round[:n].copy(),
                   host.value[:n].copy(), host.frm[:n].copy(), host.sig[:n].copy())
    model, allowed, online = host_cpu_info()
    share = min(allowed, int(os.environ.get("OMP_NUM_THREADS", allowed) or allowed))
    f = len(sigs) // 3
    pv = lambda h, r: O.canonical_value(h, r)
    figures = {}
    legs = [("all_threads", args.cpu_threads or allowed), ("per_gpu_share", share)]
    if legs[0][1] == share:
        legs = legs[1:]
    for label, threads in legs:
        t0 = time.perf_counter()
        verdict, rec = co.verify(sample, sigs, True, threads=threads)
        t1 = time.perf_counter()
        tal = co.tally(sample, verdict, f, propose_value=pv)
        t2 = time.perf_counter()
        figures[label] = {"threads": threads, "msgs_per_s": n / (t2 - t0), "verify_s": t1 - t0, "tally_decide_s": t2 - t1}
    # bit-exact check against the GPU (verdicts and signatories of the timed
    # run; the GPU tally of the same sample with the GPU's verdicts)
    gv = gpu_verdict[:n].cpu().numpy()
    exact_verify = verdict.tolist() == gv.tolist() and rec.tobytes() == gpu_recovered[:n].cpu().numpy().tobytes()
    gt = v.tally(sample, gv)
    c_counts = {(int(h), int(r), int(t), sample.value[rep].tobytes()): int(k) for h, r, t, rep, k in tal["counts"]}
    c_any = {(int(h), int(r)): int(a) for h, r, _, _, a, _ in tal["hr"]}
    bits = ("timeout_prevote", "precommit_nil", "timeout_precommit_reached", "timeout_precommit_exact", "skip",
            "precommit_value", "commit")
    dec_ok = all({k: bool(d >> j & 1) for j, k in enumerate(bits)} ==
                 {k: quorum.decide(gt, int(h), int(r), f, pv(int(h), int(r)), True)[k] for k in bits}
                 for (h, r), d in zip(tal["hr"][:, :2].tolist(), tal["decide"].tolist()))
    exact_tally = c_counts == gt.count and c_any == gt.distinct_any
    best = max(figures.values(), key=lambda fig: fig["msgs_per_s"])
    glv = {}
    try:
        gp = glv_port()
        threads = best["threads"]
        t0 = time.perf_counter()
        gverdict, grec = gp.verify(sample, sigs, True, threads=threads)
        t1 = time.perf_counter()
        co.tally(sample, gverdict, f, propose_value=pv)
        t2 = time.perf_counter()
        glv = {"threads": threads, "msgs_per_s": n / (t2 - t0), "verify_s": t1 - t0, "tally_decide_s": t2 - t1,
               "bit_exact_vs_gpu": bool(gverdict.tolist() == gv.tolist()
                                        and grec.tobytes() == gpu_recovered[:n].cpu().numpy().tobytes())}
    except Exception as e:  # reported, never fatal
        glv = {"error": repr(e)}
    try:
        sp = secp_port()
        threads = best["threads"]
        t0 = time.perf_counter()
        sverdict, srec = sp.verify(sample, sigs, True, threads=threads)
        t1 = time.perf_counter()
        co.tally(sample, sverdict, f, propose_value=pv)
        t2 = time.perf_counter()
        secp = {"threads": threads, "msgs_per_s": n / (t2 - t0), "verify_s": t1 - t0, "tally_decide_s": t2 - t1,
                "bit_exact_vs_gpu": bool(sverdict.tolist() == gv.tolist()
                                         and srec.tobytes() == gpu_recovered[:n].cpu().numpy().tobytes()),
                "note": "C++ restatement, not Go: 5 x 52-bit field, GLV + wNAF Strauss ladder (wNAF-5 R, "
                        "wNAF-15 over 8,192 precomputed odd multiples of G), 62-bit divstep inversions"}
    except Exception as e:  # reported, never fatal
        secp = {"error": repr(e)}
    kind, value, cores = "port", best["msgs_per_s"], best["threads"]
    if glv.get("msgs_per_s", 0) > value and glv.get("bit_exact_vs_gpu"):
        kind, value, cores = "port-glv", glv["msgs_per_s"], glv["threads"]
    if secp.get("msgs_per_s", 0) > value and secp.get("bit_exact_vs_gpu"):
        kind, value, cores = "port-secp-class", secp["msgs_per_s"], secp["threads"]
    chosen = {"port": best, "port-glv": glv, "port-secp-class": secp}[kind]
    # "kind" keeps the contract's vocabulary ("port": a restatement, not the
    # reference's own code); "port_name" says which of the three ports it is
    return {"value": value, "unit": "msgs/s", "cores": cores, "kind": "port", "port_name": kind,
            "verify_s": chosen["verify_s"], "tally_decide_s": chosen["tally_decide_s"],
            "port_secp_class": secp, "port_glv": glv,
            "port_naive": {"msgs_per_s": best["msgs_per_s"], "threads": best["threads"], "by_threads": figures},
            "cpu_model": model, "host_cpus_allowed": allowed, "host_cpus_online": online,
            "cgroup_cpu_quota": cgroup_cpu_quota(),
            "value_from": (f"'{kind}' on {cores} threads: the fastest of the three host ports that is bit-exact "
                           f"with the GPU; all three run on the thread count at which the naive port was faster "
                           f"(" + ", ".join(f"{k} {fig['threads']}" for k, fig in figures.items()) + ")"),
            "bit_exact_vs_gpu": bool(exact_verify and exact_tally and dec_ok),
            "bit_exact_detail": {"verdicts_and_signatories": bool(exact_verify), "tally_rows": bool(exact_tally),
                                 "decisions": bool(dec_ok), "rounds_decided": int(len(tal["hr"])),
                                 "commits": int(sum(d >> 6 & 1 for d in tal["decide"].tolist()))},
            "sample": f"first {n} messages of the same C2 workload: verify (digest+recover+signatory+membership) "
                      f"on the host threads, then the first-wins tally and every round's quorum decisions",
            "note": "value = the fastest of three bit-exact host ports: 'port' is the C restatement with naive "
                    "4x64-bit-limb arithmetic (no GLV, no tables); 'port-glv' is the repository's own recovery "
                    "(GLV split, 12-bit G / lambda G tables, divstep inversions) built for the host, whose "
                    "radix-2^29 limbs suit the GPU's 32-bit multiplier rather than the host's 64-bit one; "
                    "'port-secp-class' (oracle/secp_port.cpp) restates the path in libsecp256k1's algorithm "
                    "class (5 x 52-bit field, GLV + wNAF, precomputed G table, 62-bit divsteps).  libsecp256k1 "
                    "itself, which the reference reaches through go-ethereum's cgo, cannot be built here "
                    "(C++ restatement, not Go)",
            "valid": int((verdict == 0).sum())}


if __name__ == "__main__":
    main()
