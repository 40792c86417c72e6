"""The host-buffer (cgo) path alone: bench.py's host_buffers (hd_verify_submit /
hd_verify_submit_compact / hd_verify_wait, pinned and pageable host
batches), for a rocprofv3 --kernel-trace --memory-copy-trace run; then the
host time of each submit and wait of the compact pinned form (where the
submitting thread spends its time)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np
import torch

import bench
import hyperdrive_amd as hd
from hyperdrive_amd.device import generate
from hyperdrive_amd.verify import CompactBatch


class A:
    batch = 1 << 20
    signers = 100


dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
v = hd.Verifier(0)
sigs, foreign = v.gen_keys(100)
v.set_signatories(sigs)
print(json.dumps(bench.host_buffers(v, A, sigs, foreign, dev)), flush=True)

# per-call host time, compact pinned, 3 in flight
B = A.batch
db, _, _ = generate(v, 0, B, 100, 0, keys=(sigs, foreign), device=str(dev))
hb = db.to_host()
hb.valid_round = None
cb = CompactBatch.from_batch(hb, sigs)
keep = []


def pinned(a):
    t = torch.empty(a.shape, dtype={np.uint8: torch.uint8, np.int64: torch.int64, np.uint16: torch.int16,
                                     np.uint32: torch.int32}[a.dtype.type], pin_memory=True)
    keep.append(t)
    o = t.numpy().view(a.dtype)
    o[...] = a
    return o


src = CompactBatch(*(pinned(a) if a is not None else None for a in
                     (cb.type, cb.height, cb.round, cb.valid_round, cb.from_idx, cb.value_idx, cb.sig, cb.escape,
                      cb.values)))
outs = [(pinned(np.zeros(B, np.uint8)), pinned(np.zeros((B, 32), np.uint8))) for _ in range(3)]
for k in range(3):
    v.wait(v.submit_compact(src, *outs[k]))
sub, wai, pend = [], [], []
t0 = time.perf_counter()
for k in range(16):
    a = time.perf_counter()
    pend.append(v.submit_compact(src, *outs[k % 3]))
    sub.append(time.perf_counter() - a)
    if len(pend) == 3:
        a = time.perf_counter()
        v.wait(pend.pop(0))
        wai.append(time.perf_counter() - a)
for t in pend:
    v.wait(t)
dt = time.perf_counter() - t0
print(json.dumps({"compact_pinned_msgs_per_s": B * 16 / dt, "ms_per_batch": dt / 16 * 1e3,
                  "submit_ms": [round(x * 1e3, 3) for x in sub], "wait_ms": [round(x * 1e3, 3) for x in wai]}),
      flush=True)
