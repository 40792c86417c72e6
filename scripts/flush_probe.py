"""Where a C5 ingress flush spends its ~50 us (bench.py ingress_c5's 64
flushes): the Ingress loop (reset_height + flush), the same consumes through
the raw foreign call with its arguments prepared once, and the host-only
parts (vote-table reset, Python result building).  Each variant runs on a
freshly pushed queue; wall times per flush in microseconds."""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np
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
    parts.append((t, marshal_device(v, t, sub, with_sig=True, stream=ws), sub.n))
ing = Ingress(v, height=1, max_capacity=1000)
os.environ["HD_MQ_MAPPED"] = "0"          # the download path, for the A/B
ing_dl = Ingress(v, height=1, max_capacity=1000)
del os.environ["HD_MQ_MAPPED"]
H = 64


def fresh(ing=ing):
    ing.height = 1
    ing.votes.reset(1)
    ing._clean = None
    ing.mq.drop_below(2 ** 62)
    ing.push_wires(parts)
    torch.cuda.synchronize()


def loop_ingress(ing=ing):
    d = 0
    for h in range(1, H + 1):
        if h > 1:
            ing.reset_height(h)
        d += len(ing.flush().consumed)
    return d


lib = ing.mq._lib
q = ing.mq._q
vt = ing.votes._v
a, snd, out = ing.mq._out_arrays(1024)
st, dbl, ev = ing.mq._vote_arrays()
got, removed, ins = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
args = (ctypes.byref(out), snd.ctypes.data, ing.mq._cap, ctypes.byref(got), ctypes.byref(removed), st.ctypes.data,
        dbl.ctypes.data, ev.ctypes.data, ctypes.byref(ins))


def loop_raw():
    d = 0
    for h in range(1, H + 1):
        if h > 1:
            lib.hd_votes_reset(vt, h)
        lib.hd_mq_consume_votes(q, vt, h, None, 0, *args)
        d += got.value
    return d


def loop_reset_only():
    for h in range(1, H + 1):
        lib.hd_votes_reset(vt, h)
    return 0


rows = []
for rep in range(4):
    rec = {}
    for name, fn in (("ingress", loop_ingress), ("raw", loop_raw), ("reset_only", loop_reset_only)):
        fresh()
        t0 = time.perf_counter()
        d = fn()
        rec[name + "_us"] = round((time.perf_counter() - t0) * 1e6 / H, 2)
        rec[name + "_delivered"] = d
    for name, fn in (("ingress_download", lambda: loop_ingress(ing_dl)),):
        fresh(ing_dl)
        t0 = time.perf_counter()
        d = fn()
        rec[name + "_us"] = round((time.perf_counter() - t0) * 1e6 / H, 2)
        rec[name + "_delivered"] = d
    rows.append(rec)
    print(json.dumps(rec), flush=True)
print(json.dumps({"flush_probe": rows}), flush=True)
