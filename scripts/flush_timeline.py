"""Per-flush host times of the C5 ingress (bench.ingress_c5's setup): for
each of 4 cycles (push, then 64 x (reset_height + flush)), the flush phase's
total and the slowest flushes, to see where a slow cycle's time goes."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

import hyperdrive_amd as hd
from hyperdrive_amd.codec import marshal_device
from hyperdrive_amd.device import DeviceBatch, generate, work_stream
from hyperdrive_amd.ingress import Ingress

dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
ws = work_stream(dev, priority=-1)
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
ing = Ingress(v, height=1, max_capacity=1000)
for _ in range(2):
    ing.push_wires([(t, wire, sub.n) for t, sub, wire in parts])
    ing.flush()
    ing.mq.drop_below(2 ** 62)
for cyc in range(4):
    ing.height = 1
    ing.votes.reset(1)
    ing._clean = None
    ing.mq.drop_below(2 ** 62)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ing.push_wires([(t, wire, sub.n) for t, sub, wire in parts])
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    per = []
    for h in range(1, 65):
        a = time.perf_counter()
        if h > 1:
            ing.reset_height(h)
        b = time.perf_counter()
        k = len(ing.flush().consumed)
        c = time.perf_counter()
        per.append((round((c - a) * 1e6, 1), round((b - a) * 1e6, 1), h, k))
    t2 = time.perf_counter()
    slow = sorted(per, reverse=True)[:6]
    med = sorted(p[0] for p in per)[32]
    print(json.dumps({"cycle": cyc, "push_ms": round((t1 - t0) * 1e3, 3), "flush_ms": round((t2 - t1) * 1e3, 3),
                      "flush_us_median": med, "slowest_us_(total,reset,h,n)": slow}), flush=True)
ing.close()
v.close()
