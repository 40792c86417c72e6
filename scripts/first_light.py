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
    assert hb.type.tolist() == ob.mtype and hb.height.tolist() == ob.height and hb.round.tolist() == ob.round
    assert hb.value.tobytes() == b"".join(ob.value) and hb.frm.tobytes() == b"".join(ob.frm)
    bad = [i for i in range(n) if hb.sig[i].tobytes() != ob.sig[i]]
    assert not bad, f"sig mismatch at {bad[:10]}"
    assert db.adv_class.cpu().numpy().tolist() == cls
    res = v.verify_batch(hb)
    vs, recs = O.verify_batch(ob, sorted(O.admitted_set(S, keys)))
    assert res.verdict.tolist() == vs, (res.verdict.tolist(), vs)
    assert res.recovered.tobytes() == b"".join(recs)
    bm = np.unpackbits(res.valid_bitmap.view(np.uint8), bitorder="little")[:n]
    assert bm.tolist() == [int(x == 0) for x in vs]
    log(f"kind {kind} n={n} adv={adv}: gen+verify parity ok; verdicts {np.bincount(res.verdict, minlength=8).tolist()}")

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
stream = torch.cuda.current_stream().cuda_stream
v.verify_batch_device(cb, verdict.data_ptr(), None, signer.data_ptr(), bitmap.data_ptr(), stream)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(3):
    v.verify_batch_device(cb, verdict.data_ptr(), None, signer.data_ptr(), bitmap.data_ptr(), stream)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 3
vc = torch.bincount(verdict.long(), minlength=8).cpu().tolist()
log(f"k_verify 1M: {ms:.2f} ms -> {N/ms*1e3/1e6:.3f} M msgs/s; verdicts {vc}")
log(json.dumps({"ms": ms, "msgs_per_s": N / ms * 1e3}))
