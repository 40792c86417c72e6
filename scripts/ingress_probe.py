"""C5 through the replica ingress, phase by phase (bench.py ingress_c5's
workload): push_wire per buffer vs push_wires (two streams), each repeated,
then the flushes.  Wall times with a device sync around each phase."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import torch

import hyperdrive_amd as hd
from hyperdrive_amd.codec import marshal_device, unmarshal_device
from hyperdrive_amd.device import DeviceBatch, generate, work_stream
from hyperdrive_amd.ingress import Ingress

dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
ws = work_stream(dev, priority=int(os.environ.get("AB_VPRIO", "-1")))
torch.cuda.set_stream(ws)
v = hd.Verifier(0)
sigs, foreign = v.gen_keys(100)
v.set_signatories(sigs)
n = 1 << 20
db, _, _ = generate(v, 0, n, 100, 30, keys=(sigs, foreign), device=str(dev))
g = torch.Generator(device=dev)
g.manual_seed(5)
perm = torch.randperm(n, device=dev, generator=g)
parts = []
for t in (2, 3):
    idx = perm[(db.type == t)[perm]]
    sub = DeviceBatch(int(idx.numel()), *(getattr(db, f)[idx].contiguous()
                                           for f in ("type", "height", "round", "valid_round", "value", "frm", "sig")))
    parts.append((t, sub, marshal_device(v, t, sub, with_sig=True, stream=ws)))
v.verify_batch_device(db.c_struct(), torch.empty(n, dtype=torch.uint8, device=dev).data_ptr(), None, None, None,
                      ws.cuda_stream)                                     # learn the keys
torch.cuda.synchronize()
out = {}


def clock(fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = fn()
    torch.cuda.synchronize()
    return r, (time.perf_counter() - t0) * 1e3


ing = Ingress(v, height=1, max_capacity=1000)
rows = []
for rep in range(3):
    ing.votes.reset(1)
    ing.mq.drop_below(2 ** 62)
    rec = {}
    # phases of push_wire, one buffer after the other
    for t, sub, wire in parts:
        (dbu, _), rec[f"unmarshal_{t}"] = clock(lambda: unmarshal_device(v, t, wire, sub.n, True, stream=ws))
        verdict = torch.empty(sub.n, dtype=torch.uint8, device=dev)
        _, rec[f"verify_{t}"] = clock(lambda: v.verify_batch_device(dbu.c_struct(), verdict.data_ptr(), None, None,
                                                                    None, ws.cuda_stream))
        _, rec[f"insert_{t}"] = clock(lambda: ing.mq.insert_verified_device(dbu, verdict, 1, stream=ws))
        for k in range(2):      # authentication only (the ingress's call); the second run sizes by the first
            _, rec[f"auth_{t}"] = clock(lambda: v.authenticate_batch_device(dbu.c_struct(), verdict.data_ptr(),
                                                                          ws.cuda_stream))
        rec[f"auth_fallback_{t}"] = v.fastpath_stats()[1]
        for k in range(2):
            _, rec[f"verify2_{t}"] = clock(lambda: v.verify_batch_device(dbu.c_struct(), verdict.data_ptr(), None,
                                                                       None, None, ws.cuda_stream))
        rec[f"verify_fallback_{t}"] = v.fastpath_stats()[1]
    ing.mq.drop_below(2 ** 62)
    _, rec["push_wire_x2"] = clock(lambda: [ing.push_wire(t, wire, sub.n, stream=ws) for t, sub, wire in parts])
    for k in range(3):          # interleaved A/B of the fallback's wave priority (HD_VAR_WAVE_PRIO)
        for prio in (0, 2):
            v.set_variant("wave_prio", prio)
            ing.mq.drop_below(2 ** 62)
            _, rec[f"push_wires_prio{prio}_{k}"] = clock(
                lambda: ing.push_wires([(t, wire, sub.n) for t, sub, wire in parts]))
    v.set_variant("wave_prio", 0)
    ing.mq.drop_below(2 ** 62)
    _, rec["push_wires"] = clock(lambda: ing.push_wires([(t, wire, sub.n) for t, sub, wire in parts]))
    t0 = time.perf_counter()
    delivered = 0
    for h in range(1, 65):
        if h > 1:
            ing.reset_height(h)
        delivered += len(ing.flush().consumed)
    rec["flush64"] = (time.perf_counter() - t0) * 1e3
    rec["delivered"] = delivered
    ing.height = 1
    rows.append({k: round(x, 3) if isinstance(x, float) else x for k, x in rec.items()})
print(json.dumps({"ingress_c5_phases_ms": rows}), flush=True)
