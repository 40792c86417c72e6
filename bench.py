#!/usr/bin/env python3
"""Benchmark: verified consensus msgs/s (secp256k1) on MI355X.

Workload (BASELINE.json configs[1]): batch-verify 1,048,576 synthetic
Prevote/Precommit messages from 100 signatories per GPU (SURVEY §8(d) C2:
signer = i % 100, type = 2 + (i/100)%2, h = 1 + i/200, r = 0; 90 % canonical
value, 5 % nil, 5 % random), seeded, signed with RFC6979 on the GPU before the
timed region.  One step = the hot path over one batch: k_verify (digest ->
recover -> signatory -> Equal(From) -> admitted) over this rank's shard, the
valid-bitmap all-gather over RCCL (N > 1), and the first-wins 2f+1 tally of
the whole batch.  Inputs are resident in HBM when timing starts.

Multi-GPU: one process per GPU (torch.distributed.run), weak scaling: rank k
verifies messages [k*B, (k+1)*B) of the N*B-message stream (C4 generator);
the batch metadata is replicated, only the verdict bitmaps cross xGMI.

Prints ONE JSON line on rank 0.  The CPU baseline is the C restatement of the
same path (oracle/hd_oracle.c) on the host's cores over a bounded sample.
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
# the rest mixed additions (8M + 3S each); s^-1 mod n (296 M, as SURVEY's
# r^-1) and Z^-1 mod p (274 M) once per `per_inv` messages; Montgomery's trick
# (3 M per message and kind), u1 and u2 (2 M), the affine comparison (1S + 3M);
# one SHA-256 compression (2,200 ops).
M_OPS = 160


def fast_ops_per_msg(g_windows, key_windows, per_inv):
    adds = g_windows + key_windows - 1
    return (adds * 11 + (296 + 274) / per_inv + 2 * 3 + 2 + 4) * M_OPS + 2200


BYTES_PER_MSG = 146 + 33        # HBM in + out per message
# INT32 VALU peak of one MI355X: 256 CU x 4 SIMD x 32 lanes x 2.4 GHz (the
# FP32-vector issue rate of MI355X_MICROARCH.md, 157.3 TFLOPS / 2 per FMA)
VALU_PEAK_OPS = 256 * 4 * 32 * 2.4e9


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=1 << 20, help="messages per GPU")
    ap.add_argument("--signers", type=int, default=100)
    ap.add_argument("--adv", type=int, default=0, help="adversarial percentage (C5)")
    ap.add_argument("--cpu-sample", type=int, default=1 << 20,
                    help="messages of the CPU-baseline sample (~8 s on 16 host threads)")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-tally", action="store_true")
    ap.add_argument("--no-aux", action="store_true", help="skip the SURVEY §8(f) side measurements")
    return ap.parse_args()


def cpu_baseline(args, S):
    """C restatement of the reference path on the host cores (bounded sample)."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import subprocess
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    from oracle_c import COracle
    co = COracle(os.path.join(ROOT, "oracle", "_build", "liboracle.so"))
    return co


def main():
    args = parse()
    import numpy as np
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        dist = None
        torch.cuda.set_device(0)
    dev = torch.device("cuda", local if world > 1 else 0)

    import hyperdrive_amd as hd
    from hyperdrive_amd import _lib
    from hyperdrive_amd.device import DeviceBatch, generate
    from hyperdrive_amd._lib import HdBatch

    B, S = args.batch, args.signers
    total = B * world
    v = hd.Verifier(dev.index)
    sigs, foreign = v.gen_keys(S)
    v.set_signatories(sigs)
    t0 = time.time()
    # replicated batch metadata (whole stream), generated on this GPU
    db, _, _ = generate(v, 0, total, S, args.adv, keys=(sigs, foreign), device=str(dev))
    gen_s = time.time() - t0

    from hyperdrive_amd.device import work_stream
    ws = work_stream(dev)
    torch.cuda.set_stream(ws)          # torch ops (RCCL all-gather included) share the library's stream
    stream = ws.cuda_stream
    from hyperdrive_amd.shard import gather_bitmaps, shard_range
    lo, hi = shard_range(total, rank, world)
    assert hi - lo == B
    # shard views (device pointers offset into the replicated batch)
    shard = HdBatch(B, db.type.data_ptr() + lo, db.height.data_ptr() + 8 * lo, db.round.data_ptr() + 8 * lo,
                    db.valid_round.data_ptr() + 8 * lo, db.value.data_ptr() + 32 * lo, db.frm.data_ptr() + 32 * lo,
                    db.sig.data_ptr() + 65 * lo)
    full = db.c_struct()
    assert B % 32 == 0
    # triple-buffered outputs: the tally of step k (its own stream; the call
    # returns once its host outputs are complete) runs while the verifications
    # of steps k+1 and k+2 are queued, so a slow host sync never drains the
    # verify queue; every step's verify and tally complete inside the timed
    # region
    NBUF = 3
    verdicts = [torch.empty(B, dtype=torch.uint8, device=dev) for _ in range(NBUF)]
    bitmaps = [torch.zeros(B // 32, dtype=torch.int32, device=dev) for _ in range(NBUF)]
    lib = _lib.load()
    t_out, t_arr = v._tally_struct(total)
    ts = torch.cuda.Stream(device=dev)

    ev_k = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    tally_info = {}

    def verify(k, record=False):
        buf = k % NBUF
        if record:
            ev_k[k][0].record(ws)
        v.verify_batch_device(shard, verdicts[buf].data_ptr(), None, None, bitmaps[buf].data_ptr(), stream)
        if record:
            ev_k[k][1].record(ws)
        if dist is not None:
            gathered = gather_bitmaps(bitmaps[buf], total, world)   # RCCL all-gather over xGMI
        else:
            gathered = bitmaps[buf]
        done = torch.cuda.Event()
        done.record(ws)
        return gathered, done

    def tally(pending):
        if pending is None or args.no_tally:
            return
        gathered, done = pending
        ts.wait_event(done)
        rc = lib.hd_tally_device_bitmap(v.handle, ctypes.byref(full), gathered.data_ptr(), ctypes.byref(t_out),
                                        ts.cuda_stream)
        if rc != 0:
            raise _lib.HDError(rc, "hd_tally_device_bitmap", lib.hd_ctx_last_error(v.handle).decode())
        tally_info["n_hr"] = t_out.n_hr
        tally_info["n_counts"] = t_out.n_counts

    def run(steps, record):
        # buffer k % NBUF is rewritten by verify(k + NBUF), queued only after
        # tally(k) has returned (hd_tally_device_bitmap synchronises its stream)
        pending = []
        for k in range(steps):
            pending.append(verify(k, record))
            if len(pending) == NBUF:
                tally(pending.pop(0))
        while pending:
            tally(pending.pop(0))

    # context setup, outside the timed region (like the generator tables): one
    # verification of this rank's shard teaches the context the keys of the
    # signatories (their first VALID full recovery) and builds their
    # fixed-base tables -- a long-lived replica has them from earlier batches.
    # Every timed step still verifies every message.
    # The same pass primes the tally's device tables, so even --warmup 0
    # times steady-state steps.
    t_setup = time.time()
    run(1, False)
    torch.cuda.synchronize(dev)
    setup_s = time.time() - t_setup
    run(args.warmup, False)
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t_start = time.perf_counter()
    run(args.steps, True)
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t_start
    kernel_ms = [a.elapsed_time(b) for a, b in ev_k]
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    verdict, bitmap = verdicts[(args.steps - 1) % 2], bitmaps[(args.steps - 1) % 2]

    # correctness gate: without --adv every message of the workload is an honest
    # vote by construction, so every verdict must be VALID and the valid bitmap
    # full; a wrong kernel must not produce a throughput number.
    hist = torch.bincount(verdict.long(), minlength=8).cpu().tolist()
    if args.adv == 0:
        full_bits = int(bitmap.view(torch.uint8).cpu().numpy().astype("uint8").sum())
        if hist[0] != B or full_bits != 255 * (B // 8):
            print(json.dumps({"error": "verification produced wrong verdicts", "verdicts": hist}), flush=True)
            sys.exit(1)

    if rank == 0:
        ms_step = elapsed / args.steps * 1e3
        value = total * args.steps / elapsed
        k_ms = sum(kernel_ms) / len(kernel_ms)
        known, fallback = v.fastpath_stats()
        # messages of the last step by path: full recovery for `fallback`,
        # the known-key check for the rest
        geom = v.fastpath_geometry()
        w_fast = fast_ops_per_msg(*geom)
        if os.environ.get("HD_VERIFY_FASTPATH", "1") == "0":
            fallback = B                 # fast path off: every message takes the full recovery
        w_msg = ((B - fallback) * w_fast + fallback * W_OPS_PER_MSG) / B
        achieved = B * w_msg / (k_ms * 1e-3)
        out = {
            "metric": "verified consensus msgs/sec (secp256k1) at 1/2/4/8 MI355X; % INT32 VALU peak",
            "value": value,
            "unit": "msgs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32 (256-bit modular integer arithmetic)",
            "data": "synthetic (seeded RFC6979-signed votes generated on the GPU)",
            "config": {"workload": "C2: batch-verify 1M Prevote/Precommit from 100 signatories + 2f+1 tally",
                       "messages_per_gpu": B, "global_batch": total, "signatories": S, "adversarial_pct": args.adv,
                       "parallelism": f"shard-by-index x{world}, RCCL all-gather of valid bitmaps"},
            "roofline": {
                "bound": "valu",
                "kernel": "verify call: k_fast_scalars + k_fast_sums + k_fast_final (known-key check), "
                          "k_verify on the fallback list",
                "achieved": achieved / 1e12,
                "peak": VALU_PEAK_OPS / 1e12,
                "unit": "TOP/s (int32 lane-ops)",
                "frac": achieved / VALU_PEAK_OPS,
                "traffic": (pmc_traffic() or {}).get("bytes_per_launch_corrected"),
                "traffic_detail": pmc_traffic(),
                "kernel_ms": k_ms,
                "algorithmic_ops_per_msg": w_msg,
                "ops_model": {"known_key_check": w_fast, "full_recovery": W_OPS_PER_MSG,
                              "geometry": {"g_windows": geom[0], "key_windows": geom[1], "msgs_per_inversion": geom[2]},
                              "fallback_msgs_last_step": fallback, "known_signatories": known},
                "hbm_algorithmic_GBs": B * BYTES_PER_MSG / (k_ms * 1e-3) / 1e9,
            },
            "verdicts": hist,
            "tally": tally_info,
            "gen_s": gen_s,
            "key_setup_s": setup_s,
        }
        # aux rows and the CPU baseline: single-GPU runs only (the N>1 runs
        # report the sharded headline path; other ranks wait at the barrier)
        if not args.no_aux and world == 1:
            try:
                out["aux"] = aux_benchmarks(v, db, ws)
            except Exception as e:  # reported, never fatal for the headline number
                out["aux"] = {"error": repr(e)}
        if not args.no_cpu and world == 1:
            try:
                out["cpu_baseline"] = run_cpu_baseline(args, db, sigs)
            except Exception as e:  # reported, never fatal for the GPU number
                out["cpu_baseline"] = {"error": repr(e)}
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


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
    ing.reset_height(1)
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
    """HBM bytes per verify call of the known-key check from the committed
    rocprofv3 PMC passes (profiles/round1/pmc_known_key_check.json: FETCH_SIZE +
    WRITE_SIZE of k_fast_scalars, k_fast_sums and k_fast_final, separate
    passes, KiB -> bytes; FETCH_SIZE doubled per MI355X_MICROARCH.md's gfx950
    correction).  The table reads (24 x 72 B per message) dominate; the batch
    itself is 179 B/message and the rows between the kernels ~0.5 kB."""
    path = os.path.join(ROOT, "profiles", "round1", "pmc_known_key_check.json")
    try:
        with open(path) as fh:
            p = json.load(fh)
        return {"bytes_per_launch_raw": p["hbm_bytes_raw"], "bytes_per_launch_corrected": p["hbm_bytes_corrected"],
                "source": "profiles/round1/pmc_known_key_check.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE)"}
    except (OSError, KeyError, ValueError):
        return None


def run_cpu_baseline(args, db, sigs):
    """Time the C restatement (oracle/hd_oracle.c, kind 'port') on host threads
    over the first --cpu-sample messages of the same workload."""
    import numpy as np
    co = cpu_baseline(args, None)
    n = min(args.cpu_sample, db.n)
    host = db.to_host()
    from hyperdrive_amd.verify import Batch
    sample = Batch(host.type[:n].copy(), host.height[:n].copy(), host.round[:n].copy(), host.valid_round[:n].copy(),
                   host.value[:n].copy(), host.frm[:n].copy(), host.sig[:n].copy())
    threads = args.cpu_threads
    t = time.perf_counter()
    verdict, _ = co.verify(sample, sigs, True, threads=threads)
    dt = time.perf_counter() - t
    return {"value": n / dt, "unit": "msgs/s", "cores": threads, "kind": "port",
            "sample": f"first {n} messages of the same C2 workload, verify path (digest+recover+signatory+"
                      f"membership) of oracle/hd_oracle.c on {threads} host threads",
            "wall_s": dt, "valid": int((verdict == 0).sum())}


if __name__ == "__main__":
    main()
