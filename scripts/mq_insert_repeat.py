"""The 1M insert of test_million_message_insert repeated REPS times (default
3), each against the numpy restatement, with a diagnosis of the first
mismatch (messages dropped, or reordered)."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import hyperdrive_amd as hd
from hyperdrive_amd.device import DeviceBatch
from hyperdrive_amd.mq import MessageQueue

v = hd.Verifier(0)
rng = np.random.default_rng(11)
n, S = 1 << 20, 100
h = rng.integers(1, 5000, n).astype(np.int64)
r = rng.integers(0, 4, n).astype(np.int64)
snd = (np.arange(n) % S).astype(np.int32)
keys = rng.integers(0, 256, (S, 32), dtype=np.uint8)
t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
tag = np.zeros((n, 32), np.uint8)
tag[:, :4] = np.arange(n, dtype=np.uint32).view(np.uint8).reshape(n, 4)
db = DeviceBatch(n, t(np.full(n, 2, np.uint8)), t(h), t(r), t(np.full(n, -1, np.int64)), t(tag),
                 t(keys[snd]), t(np.zeros((n, 65), np.uint8)))
order = np.lexsort((np.arange(n), r, h, snd))
keep = np.concatenate([order[snd[order] == k][:1000] for k in range(S)])
for rep in range(int(os.environ.get("REPS", "3"))):
    q = MessageQueue(v, 1000)
    q.insert_device(db)
    b, s = q.consume(10 ** 9, keys)
    idx = b.value[:, :4].copy().view(np.uint32).ravel().astype(np.int64)
    ok = len(idx) == len(keep) and (idx == keep).all()
    print("rep", rep, "len", len(idx), "ok", ok, flush=True)
    if not ok:
        d = np.nonzero(idx[:len(keep)] != keep[:len(idx)])[0]
        print(" mismatches", len(d), "first", d[:5].tolist())
        missing = np.setdiff1d(keep, idx).tolist()
        extra = np.setdiff1d(idx, keep).tolist()
        print(" missing", len(missing), missing[:10], "extra", len(extra), extra[:10])
        for e in missing[:5]:
            print("  missing", e, "snd", snd[e], "h", h[e], "r", r[e])
        same_set = len(missing) == 0
        if same_set:
            i = d[0]
            print("  reordered at", i, [(int(x), int(h[x]), int(r[x])) for x in idx[i - 2:i + 3]])
            print("  want        ", [(int(x), int(h[x]), int(r[x])) for x in keep[i - 2:i + 3]])
    q.close()
v.close()
