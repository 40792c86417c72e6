"""Deterministic reproducer of the round-4 routed-tally mismatch
(test_multi_gpu.py test_routed_kernels_match_restatement[8]).

The round-4 test passed torch.cuda.current_stream().cuda_stream to the
library.  Torch's default stream has handle 0, and the C ABI reads a NULL
stream as the context's own stream, which is created non-blocking: it is not
ordered after torch's work on the legacy NULL stream.  So hd_unroute_device
could read the received-rows tensor before torch.cat had written it.

Here a ~20 ms sleep kernel sits on torch's stream in front of the torch.cat,
which makes that window certain:
  mode "null":     the round-4 flow (stream 0 everywhere)  -> owners' tallies
                   differ from the restatement (rows read before they exist)
  mode "explicit": one explicit stream for torch and the library -> equal

    python scripts/null_stream_race.py
(A diagnostic; reads tests/ restatements, so it is not shipped.)"""
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
from hyperdrive_amd.device import DeviceBatch, generate, work_stream
from hyperdrive_amd.shard import route_candidates, shard_range, tally_out, tally_routed_device, unroute
from test_multi_rank import routed_tally_rows
from util import from_np


def run(mode, world=8):
    v = hd.Verifier(0)
    S, n = 50, 20_000 + 13
    ks = v.gen_keys(S)
    v.set_signatories(ks[0])
    db, _, _ = generate(v, 0, n, S, 30, keys=ks, start=99)
    hb = db.to_host()
    res, _ = v.process_batch(hb)
    adm = sorted(bytes(x) for x in ks[0])
    ws = work_stream() if mode == "explicit" else torch.cuda.default_stream()
    cs = ws.cuda_stream
    out = []
    with torch.cuda.stream(ws):
        bits = torch.from_numpy(res.valid_bitmap.view(np.int32).copy()).cuda()
        sent = {}
        for k in range(world):
            lo, hi = shard_range(n, k, world)
            sub = DeviceBatch(hi - lo, db.type[lo:hi], db.height[lo:hi], db.round[lo:hi], db.valid_round[lo:hi],
                              db.value[lo:hi], db.frm[lo:hi], db.sig[lo:hi])
            rows, counts = route_candidates(v, sub.c_struct(), bits.data_ptr() + 4 * (lo // 32), lo, world, cs)
            torch.cuda.synchronize()            # isolate the unroute's read from the route's write
            off = np.concatenate([[0], np.cumsum(counts)])
            for o in range(world):
                sent[(k, o)] = rows[off[o]: off[o + 1]]
        for o in range(world):
            torch.cuda._sleep(50_000_000)       # torch's stream busy ~20 ms before the concatenation
            recv = torch.cat([sent[(k, o)] for k in range(world)]).contiguous()
            rb, gidx = unroute(v, recv, cs)     # cs == 0: the context's non-blocking stream
            local = tally_routed_device(v, rb, gidx, cs, tally_out(v, n, pinned=True), "cpu")
            torch.cuda.synchronize()
            want = routed_tally_rows(recv.cpu().numpy(), adm)
            got_c, want_c = local["counts"].tolist(), want["counts"].tolist()
            first = next((i for i, (a, b) in enumerate(zip(got_c, want_c)) if a != b), None)
            out.append({"owner": o, "rows": int(recv.shape[0]), "equal": got_c == want_c,
                        "votes": int(sum(r[4] for r in got_c)), "want_votes": int(sum(r[4] for r in want_c)),
                        "first_diff": None if first is None else {"got": got_c[first], "want": want_c[first]}})
    v.close()
    return out


if __name__ == "__main__":
    for mode in ("null", "explicit"):
        owners = run(mode)
        print(json.dumps({"mode": mode, "owners_equal": sum(o["equal"] for o in owners), "owners": len(owners),
                          "detail": owners}), flush=True)
