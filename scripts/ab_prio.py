"""A/B of context variants x verify streams, interleaved in one process,
through bench.py's Pipeline (verify + tally): C2 (1M, 100 signatories), C5
(30 % adversarial) and C3 (1000 signatories, 128,064 messages).  Prints one
JSON line per workload: ms/step per setting and round.

AB_VARS="wave_prio=0,3;split_k=-1,8" (Verifier.VARIANTS names; every
combination), AB_STREAMS="1,2"."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import torch

import bench
import hyperdrive_amd as hd
from hyperdrive_amd.device import generate, work_stream

import itertools

VARS = [(kv.split("=")[0], [int(x) for x in kv.split("=")[1].split(",")])
        for kv in os.environ.get("AB_VARS", "wave_prio=0,3").split(";") if kv]
COMBOS = list(itertools.product(*[[(k, x) for x in vals] for k, vals in VARS]))
STREAMS = [int(p) for p in os.environ.get("AB_STREAMS", "1,2").split(",")]
TALLY = os.environ.get("AB_TALLY", "on").split(",")      # on, off, nodup
ROUNDS = int(os.environ.get("AB_ROUNDS", "3"))
STEPS = int(os.environ.get("AB_STEPS", "20"))
which = sys.argv[1:] or ["C2", "C5", "C3"]

dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
ws = work_stream(dev, priority=int(os.environ.get("AB_VPRIO", "-1")))
torch.cuda.set_stream(ws)
ts = torch.cuda.Stream(device=dev, priority=0)


def ab(name, v, db, n):
    pipe = bench.Pipeline(v, db, n, 0, 0, 1, None, ws, ts)
    extra = [torch.cuda.Stream(device=dev, priority=ws.priority) for _ in range(max(STREAMS) - 1)]
    pipe.run(3)
    label = lambda combo, s, t: "_".join(f"{k}{x}" for k, x in combo) + f"_s{s}_t{t}"
    res = {label(c, s, t): [] for c in COMBOS for s in STREAMS for t in TALLY}
    dup = pipe.t_out.dup
    for _ in range(ROUNDS):
        for combo in COMBOS:
            for k, x in combo:
                v.set_variant(k, x)
            for s in STREAMS:
                for t in TALLY:
                    pipe.wss = [ws] + extra[: s - 1]
                    pipe.do_tally = t != "off"
                    pipe.t_out.dup = dup if t == "on" else None
                    pipe.run(2)
                    el = bench.timed(pipe, STEPS, None, dev)
                    res[label(combo, s, t)].append(round(el / STEPS * 1e3, 4))
    pipe.do_tally, pipe.t_out.dup = True, dup
    for k, vals in VARS:
        v.set_variant(k, vals[0])
    vd, _, _ = pipe.last(STEPS)
    hist = torch.bincount(vd.long(), minlength=8).cpu().tolist()
    best = {k: round(n / min(x) * 1e-3, 1) for k, x in res.items()}
    print(json.dumps({"workload": name, "messages": n, "ms_per_step": res, "best_M_msgs_per_s": best,
                      "verdicts": hist}), flush=True)


v = hd.Verifier(0)
sigs, foreign = v.gen_keys(100)
v.set_signatories(sigs)
B = 1 << 20
if "C2" in which:
    db, _, _ = generate(v, 0, B, 100, 0, keys=(sigs, foreign), device=str(dev))
    ab("C2", v, db, B)
    del db
if "C5" in which:
    db, _, _ = generate(v, 0, B, 100, 30, keys=(sigs, foreign), device=str(dev))
    ab("C5", v, db, B)
    del db
if "C3" in which:
    v.close()
    v3 = hd.Verifier(0)
    k3 = v3.gen_keys(1000)
    v3.set_signatories(k3[0])
    n3 = (64 * 2001 + 31) // 32 * 32
    db3, _, _ = generate(v3, 1, n3, 1000, 0, keys=k3, device=str(dev))
    ab("C3", v3, db3, n3)
