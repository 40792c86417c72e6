"""Probe for the intermittent mismatch of tests/test_multi_gpu.py
test_routed_kernels_match_restatement[8]: the same routed flow (8 owners of a
20,013-message adversarial batch on one GPU), repeated in one process.  Per
owner it checks the unrouted batch against the restatement (unroute_np), then
tallies it twice and compares both tallies with the restatement, so a
mismatch says which step went wrong and whether it repeats.

    python tests/routed_flake_probe.py [reps]

(A diagnostic, not collected by pytest: it lives under tests/ because it
checks against the oracle's restatements.)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np
import torch

import hyperdrive_amd as hd
from hyperdrive_amd.device import DeviceBatch, generate
from hyperdrive_amd.shard import route_candidates, shard_range, tally_out, tally_routed_device, unroute
from test_multi_rank import route_rows_np, routed_tally_rows, unroute_np
from util import from_np

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
world = 8
cs = torch.cuda.current_stream().cuda_stream
bad = 0
for rep in range(reps):
    v = hd.Verifier(0)
    S, n = 50, 20_000 + 13
    ks = v.gen_keys(S)
    v.set_signatories(ks[0])
    db, _, _ = generate(v, 0, n, S, 30, keys=ks, start=99)
    hb = db.to_host()
    res, _ = v.process_batch(hb)
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
        got = rows[: sum(counts)].cpu().numpy()
        if counts != want_counts or got.tobytes() != want.tobytes():
            print(json.dumps({"rep": rep, "shard": k, "route_rows_differ": True}), flush=True)
        off = np.concatenate([[0], np.cumsum(counts)])
        for o in range(world):
            sent[(k, o)] = rows[off[o]: off[o + 1]]
    for o in range(world):
        recv = torch.cat([sent[(k, o)] for k in range(world)]).contiguous()
        rnp = recv.cpu().numpy()
        rb, gidx = unroute(v, recv, cs)
        torch.cuda.synchronize()
        u = unroute_np(rnp, adm)
        ub = {"type": rb.type.cpu().numpy(), "height": rb.height.cpu().numpy(), "round": rb.round.cpu().numpy(),
              "gidx": gidx.cpu().numpy()}
        un_ok = (ub["type"].tolist() == [x[0] for x in u] and ub["height"].tolist() == [x[1] for x in u]
                 and ub["round"].tolist() == [x[2] for x in u] and ub["gidx"].tolist() == [x[5] for x in u])
        want = routed_tally_rows(rnp, adm)
        outs = []
        for _ in range(2):
            local = tally_routed_device(v, rb, gidx, cs, tally_out(v, n, pinned=True), "cpu")
            outs.append(local["counts"].tolist() == want["counts"].tolist() and
                        local["hr"].tolist() == want["hr"].tolist())
        if not (un_ok and all(outs)):
            bad += 1
            print(json.dumps({"rep": rep, "owner": o, "m": int(recv.shape[0]), "unroute_ok": un_ok,
                              "tally_ok": outs}), flush=True)
    v.close()
print(json.dumps({"reps": reps, "bad_owner_tallies": bad}), flush=True)
