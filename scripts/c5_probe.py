"""C5 sub-line stability probe: bench.py's headline context (C2, 100
signatories) then the C5 batch (30 % adversarial) timed repeatedly, printing
ms/step, the fallback count and the known-key stats per repetition, so that a
slow first measurement (learning, table builds, queue mapping) shows itself.

    python scripts/c5_probe.py [reps] [steps]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

import bench
import hyperdrive_amd as hd
from hyperdrive_amd.device import generate, work_stream

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
ws = work_stream(dev, priority=-1)
torch.cuda.set_stream(ws)
ts = torch.cuda.Stream(device=dev, priority=0)
v = hd.Verifier(0)
sigs, foreign = v.gen_keys(100)
v.set_signatories(sigs)
B = 1 << 20
db, _, _ = generate(v, 0, B, 100, 0, keys=(sigs, foreign), device=str(dev))
p2 = bench.Pipeline(v, db, B, 0, 0, 1, None, ws, ts)
p2.run(3)
el = bench.timed(p2, steps, None, dev)
print(json.dumps({"C2_ms": round(el / steps * 1e3, 4), "stats": v.fastpath_stats()}), flush=True)
db5, _, _ = generate(v, 0, B, 100, 30, keys=(sigs, foreign), device=str(dev))
p5 = bench.Pipeline(v, db5, B, 0, 0, 1, None, ws, ts)
for r in range(reps):
    t0 = time.perf_counter()
    p5.run(2)
    torch.cuda.synchronize(dev)
    warm = time.perf_counter() - t0
    el = bench.timed(p5, steps, None, dev)
    print(json.dumps({"rep": r, "warm2_ms": round(warm * 1e3, 2), "C5_ms": round(el / steps * 1e3, 4),
                      "M_msgs_per_s": round(B * steps / el / 1e6, 1), "stats": v.fastpath_stats()}), flush=True)
