"""First GPU run: VALU probes, generator + verify parity vs the Python oracle,
and a timing of k_verify at 1M messages."""
import os, sys, time, json
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
import numpy as np, torch
import hyperdrive_amd as hd
from hyperdrive_amd.device import generate, DeviceBatch
import hd_pyoracle as O

def log(*a):
    print(*a, flush=True)

for op, name in enumerate(["v_add_u32", "v_mad_u64_u32", "v_mul_lo_u32", "v_mul_hi_u32"]):
    r = hd.probe_valu(0, op, 2000)
    log(f"probe {name}: {r/1e12:.3f} T lane-ops/s")

v = hd.Verifier(0)
S = 10
t = time.time()
sigs, foreign = v.gen_keys(S)
keys = O.KeyCache()
assert sigs.tobytes() == b"".join(O.admitted_set(S, keys)), "gen_keys mismatch"
log("gen_keys parity ok", time.time() - t)
v.set_signatories(sigs)
for kind, n, adv in [(0, 256, 60), (1, 100, 40)]:
    db, _, _ = generate(v, kind, n, S, adv, keys=(sigs, foreign))
    hb = db.to_host()
    ob, cls = O.gen_batch(kind, n, S, adv, keys=keys)
    gcls = db.adv_class.cpu().numpy().tolist()
    for i in range(n):
        f = dict(type=(int(hb.type[i]), ob.mtype[i]), h=(int(hb.height[i]), ob.height[i]), r=(int(hb.round[i]), ob.round[i]),
                 vr=(int(hb.valid_round[i]), ob.valid_round[i]), value=(hb.value[i].tobytes(), ob.value[i]),
                 frm=(hb.frm[i].tobytes(), ob.frm[i]), sig=(hb.sig[i].tobytes(), ob.sig[i]), cls=(gcls[i], cls[i]))
        badf = [k for k, (a, b) in f.items() if a != b]
        if badf:
            log(f"GEN MISMATCH kind {kind} i={i} fields {badf}: " + "; ".join(f"{k}: gpu={f[k][0]!r} ref={f[k][1]!r}" for k in badf[:3]))
            break
    else:
        log(f"kind {kind}: generator parity ok")
    # verify parity on the GPU-generated batch, oracle on the same bytes
    ob2 = O.Batch()
    for i in range(n):
        ob2.append(int(hb.type[i]), int(hb.height[i]), int(hb.round[i]), int(hb.valid_round[i]), hb.value[i].tobytes(),
                   hb.frm[i].tobytes(), hb.sig[i].tobytes())
    res = v.verify_batch(hb)
    vs, recs = O.verify_batch(ob2, sorted(O.admitted_set(S, keys)))
    assert res.verdict.tolist() == vs, (res.verdict.tolist(), vs)
    assert res.recovered.tobytes() == b"".join(recs)
    bm = np.unpackbits(res.valid_bitmap.view(np.uint8), bitorder="little")[:n]
    assert bm.tolist() == [int(x == 0) for x in vs]
    log(f"kind {kind} n={n} adv={adv}: verify parity ok; verdicts {np.bincount(res.verdict, minlength=8).tolist()}")
    vr2, tr = v.process_batch(hb)
    assert vr2.verdict.tolist() == vs
    ot = O.tally(ob2, vs)
    log("tally count eq", tr.count == ot.count, "distinct eq", tr.distinct == ot.distinct,
        "any eq", tr.distinct_any == ot.distinct_any, "dup eq", tr.dup.tolist() == ot.dup)
    if tr.count != ot.count:
        log("  gpu", sorted(tr.count.items())[:5]); log("  ref", sorted(ot.count.items())[:5])

# timing at 1M (C2)
N = 1 << 20
S = 100
sigs, foreign = v.gen_keys(S)
v.set_signatories(sigs)
t = time.time()
db, _, _ = generate(v, 0, N, S, 0, keys=(sigs, foreign))
log(f"generated {N} signed votes on GPU in {time.time()-t:.2f}s")
verdict = torch.empty(N, dtype=torch.uint8, device="cuda")
signer = torch.empty(N, dtype=torch.int32, device="cuda")
bitmap = torch.empty((N + 31) // 32, dtype=torch.int32, device="cuda")
cb = db.c_struct()
from hyperdrive_amd.device import work_stream
ws = work_stream()
stream = ws.cuda_stream
v.verify_batch_device(cb, verdict.data_ptr(), None, signer.data_ptr(), bitmap.data_ptr(), stream)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(ws)
for _ in range(3):
    v.verify_batch_device(cb, verdict.data_ptr(), None, signer.data_ptr(), bitmap.data_ptr(), stream)
e1.record(ws)
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 3
vc = torch.bincount(verdict.long(), minlength=8).cpu().tolist()
log(f"k_verify 1M: {ms:.2f} ms -> {N/ms*1e3/1e6:.3f} M msgs/s; verdicts {vc}")
log(json.dumps({"ms": ms, "msgs_per_s": N / ms * 1e3}))
