"""Host vote-log cost per flush (no GPU): hd_votes_reset + hd_votes_insert_batch
of 160 votes (a C5 ingress flush delivers ~160), through the raw foreign
call and through VoteLog.insert_batch; microseconds per flush."""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np

from hyperdrive_amd.verify import Batch
from hyperdrive_amd.votes import VoteLog

rng = np.random.default_rng(0)
n, S = 160, 100
frm = rng.integers(0, 256, (S, 32), dtype=np.uint8)
canon = rng.integers(0, 256, (1, 32), dtype=np.uint8)


def batch(h):
    t = np.where(np.arange(n) % 2 == 0, 2, 3).astype(np.uint8)
    signer = (np.arange(n) // 2) % S
    val = np.repeat(canon, n, 0)
    return Batch(t, np.full(n, h, np.int64), np.zeros(n, np.int64), np.full(n, -1, np.int64), val, frm[signer],
                 np.zeros((n, 65), np.uint8))


v = VoteLog(1)
v.set_f(33)
bs = [batch(h) for h in range(1, 65)]
lib = v._lib
st = np.zeros(n, np.uint8)
db = np.zeros(n, np.uint32)
ev = np.zeros(n, np.uint8)
ins = ctypes.c_uint32()
cs = [b.c_struct() for b in bs]
out = {}
for rep in range(3):
    t = time.perf_counter()
    for k in range(20):
        for h in range(64):
            lib.hd_votes_reset(v._v, h + 1)
            lib.hd_votes_insert_batch(v._v, ctypes.byref(cs[h]), None, st.ctypes.data, db.ctypes.data, ev.ctypes.data,
                                      ctypes.byref(ins))
    out["raw_reset_insert_us"] = (time.perf_counter() - t) / (20 * 64) * 1e6
    t = time.perf_counter()
    for k in range(20):
        for h in range(64):
            v.reset(h + 1)
            v.insert_batch(bs[h])
    out["votelog_us"] = (time.perf_counter() - t) / (20 * 64) * 1e6
    print(json.dumps(out), flush=True)
