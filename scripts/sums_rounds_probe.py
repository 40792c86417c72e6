"""k_fast_sums time per message at batch sizes that fill the chip a whole
number of times vs the headline's 1M (the tail round).

At 3 waves per SIMD the chip holds 3 x 4 x 256 = 3,072 sums waves = 768
blocks of 256 messages.  1,048,576 messages are 4,096 blocks = 5.33 rounds:
the last third-round runs one wave per SIMD.  This times the verify call and
its k_fast_sums launch (HIP events, hd_ctx_profile) on one stream for
4, 5, 5.33 and 6 rounds of the C2 stream (100 signatories, keys learned
first) and prints us per 1M messages for each: a tail that costs a full
round would show 5.33 rounds at 6/5.33 = +12.5 % per message; one that costs
nothing, equal.  One JSON line per size."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

import hyperdrive_amd as hd
from hyperdrive_amd.device import generate, work_stream

dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
ws = work_stream(dev, priority=-1)
torch.cuda.set_stream(ws)
v = hd.Verifier(0)
S = 100
ks = v.gen_keys(S)
v.set_signatories(ks[0])
BLK = 256
ROUND = 768 * BLK            # messages per full chip round at 3 waves / SIMD
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
for rounds in (4.0, 5.0, 16 / 3, 6.0, 5.0, 16 / 3):
    n = int(round(rounds * ROUND / BLK)) * BLK
    db, _, _ = generate(v, 0, n, S, 0, keys=ks, device=str(dev))
    verdict = torch.empty(n, dtype=torch.uint8, device=dev)
    bm = torch.zeros(n // 32, dtype=torch.int32, device=dev)
    for _ in range(3):        # learn / warm
        v.verify_batch_device(db.c_struct(), verdict.data_ptr(), None, None, bm.data_ptr(), ws.cuda_stream)
    ws.synchronize()
    v.profile(True)
    v.profile_read()
    for _ in range(reps):
        v.verify_batch_device(db.c_struct(), verdict.data_ptr(), None, None, bm.data_ptr(), ws.cuda_stream)
    ws.synchronize()
    calls, vms, sl, sms = v.profile_read()
    v.profile(False)
    assert int((verdict != 0).sum()) == 0
    print(json.dumps({"rounds": round(rounds, 3), "messages": n, "sums_ms": sms / sl, "call_ms": vms / calls,
                      "sums_us_per_1M": sms / sl * 1e3 * (1 << 20) / n, "call_us_per_1M": vms / calls * 1e3 * (1 << 20) / n,
                      "fallback": v.fastpath_stats()[1]}), flush=True)
    del db
v.close()
