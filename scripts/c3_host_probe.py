"""C3 host-side probe: bench.Pipeline on the C3 batch (1000 signatories,
128,064 messages) with per-call host times of the verify enqueue and of the
tally (the tally thread's foreign call: launches, one sync, the row copies),
to see whether the host threads or the device bound the step.

    python scripts/c3_host_probe.py [steps]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

import bench
import hyperdrive_amd as hd
from hyperdrive_amd.device import generate, work_stream

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 40
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
ws = work_stream(dev, priority=-1)
torch.cuda.set_stream(ws)
ts = torch.cuda.Stream(device=dev, priority=int(os.environ.get("C3_TS_PRIO", "0")))
v3 = hd.Verifier(0)
k3 = v3.gen_keys(1000)
v3.set_signatories(k3[0])
n3 = (64 * 2001 + 31) // 32 * 32
db3, _, _ = generate(v3, 1, n3, 1000, 0, keys=k3, device=str(dev))
times = {"verify": [], "tally": [], "submit": [], "collect": []}
orig_v, orig_t = bench.Pipeline.verify, bench.Pipeline.tally
orig_s, orig_c = bench.Pipeline.tally_submit, bench.Pipeline.tally_collect


def ts_(self, k, pending):
    t = time.perf_counter()
    orig_s(self, k, pending)
    times["submit"].append(time.perf_counter() - t)


def tc_(self, k):
    t = time.perf_counter()
    orig_c(self, k)
    times["collect"].append(time.perf_counter() - t)


bench.Pipeline.tally_submit, bench.Pipeline.tally_collect = ts_, tc_


def tv(self, k):
    t = time.perf_counter()
    r = orig_v(self, k)
    times["verify"].append(time.perf_counter() - t)
    return r


def tt(self, pending):
    t = time.perf_counter()
    orig_t(self, pending)
    times["tally"].append(time.perf_counter() - t)


bench.Pipeline.verify, bench.Pipeline.tally = tv, tt
for tally in (False, True):
    p = bench.Pipeline(v3, db3, n3, 0, 0, 1, None, ws, ts, tally=tally)
    p.run(4)
    torch.cuda.synchronize(dev)
    for k in times:
        times[k].clear()
    el = bench.timed(p, steps, None, dev)
    med = lambda x: sorted(x)[len(x) // 2] * 1e3 if x else None
    print(json.dumps({"tally": tally, "ms_per_step": round(el / steps * 1e3, 4),
                      "verify_enqueue_ms_median": med(times["verify"]), "tally_call_ms_median": med(times["tally"]),
                      "tally_call_ms_max": max(times["tally"]) * 1e3 if times["tally"] else None,
                      "submit_ms_median": med(times["submit"]),
                      "submit_ms_max": max(times["submit"]) * 1e3 if times["submit"] else None,
                      "collect_ms_median": med(times["collect"]),
                      "collect_ms_max": max(times["collect"]) * 1e3 if times["collect"] else None,
                      "retries": p.tally_retries}), flush=True)
