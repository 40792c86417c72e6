"""Where the cold start goes: context creation, admitted-set mapping, the first
verify calls (full recovery + key learning + table build), and the same after
a signatory-set change in a warm process."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    import torch
    import hyperdrive_amd as hd
    from hyperdrive_amd.device import generate, work_stream
    N, S = 1 << 20, 100
    out = {}
    t = time.perf_counter()
    v = hd.Verifier(0)
    torch.cuda.synchronize()
    out["ctx_create_s"] = time.perf_counter() - t
    ws = work_stream()
    verdict = torch.empty(N, dtype=torch.uint8, device="cuda")
    sigs, foreign = v.gen_keys(S)
    db, _, _ = generate(v, 0, N, S, 0, keys=(sigs, foreign))
    cb = db.c_struct()

    def calls(ver, tag):
        ms = []
        for k in range(4):
            torch.cuda.synchronize()
            t = time.perf_counter()
            ver.verify_batch_device(cb, verdict.data_ptr(), None, None, None, ws.cuda_stream)
            ws.synchronize()
            ms.append(round(time.perf_counter() - t, 4))
        out[tag + "_calls_s"] = ms
        out[tag + "_valid"] = int((verdict == 0).sum().item())

    t = time.perf_counter()
    v.set_signatories(sigs)
    torch.cuda.synchronize()
    out["set_signatories_s"] = time.perf_counter() - t
    calls(v, "fresh")
    # learned keys dropped (a pubkey-format round trip), tables kept allocated
    for fmt in (0, 1):
        v._check(v._lib.hd_ctx_set_pubkey_format(v._ctx, fmt), "set_pubkey_format")
    calls(v, "relearn")
    # a second context on the same device: allocation + learning, no G table
    t = time.perf_counter()
    v2 = hd.Verifier(0)
    v2.set_signatories(sigs)
    torch.cuda.synchronize()
    out["ctx2_create_and_set_s"] = time.perf_counter() - t
    calls(v2, "ctx2")
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
