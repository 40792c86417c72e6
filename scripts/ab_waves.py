"""A/B of k_verify register budgets (waves/SIMD) in one process, interleaved."""
import os, sys, json
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import torch
import hyperdrive_amd as hd
from hyperdrive_amd.device import generate, work_stream

N, S = 1 << 20, 100
ctxs = {}
for w in (2, 3):   # (4: the build miscompiles the recovery, removed in round 2b)
    os.environ["HD_VERIFY_WAVES"] = str(w)
    ctxs[w] = hd.Verifier(0)
sigs, foreign = ctxs[2].gen_keys(S)
for v in ctxs.values():
    v.set_signatories(sigs)
db, _, _ = generate(ctxs[2], 0, N, S, 0, keys=(sigs, foreign))
ws = work_stream()
verdict = torch.empty(N, dtype=torch.uint8, device="cuda")
cb = db.c_struct()
res = {w: [] for w in ctxs}
for rnd in range(4):
    for w, v in ctxs.items():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(ws)
        v.verify_batch_device(cb, verdict.data_ptr(), None, None, None, ws.cuda_stream)
        e1.record(ws)
        e1.synchronize()
        ok = int((verdict == 0).sum()) == N
        res[w].append(round(e0.elapsed_time(e1), 3) if ok else "WRONG")
        verdict.fill_(9)
print(json.dumps({"ms": res, "best_msgs_per_s": {w: N / min(x for x in r if x != "WRONG") * 1e3 for w, r in res.items() if any(x != "WRONG" for x in r)}}))
