"""bench.py's C5-through-ingress sub-line on its own (for a kernel trace:
rocprofv3 --kernel-trace -- python3 scripts/ingress_c5_run.py)."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

import bench
import hyperdrive_amd as hd
from hyperdrive_amd.device import work_stream

dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
ws = work_stream(dev, priority=-1)
torch.cuda.set_stream(ws)
v = hd.Verifier(0)
sigs, foreign = v.gen_keys(100)
v.set_signatories(sigs)
r = bench.ingress_c5(v, (sigs, foreign), 100, 1 << 20, ws, str(dev))
r.pop("note", None)
r["foreign_stats"] = v.foreign_stats(checks=True)
print(json.dumps(r), flush=True)
v.close()
