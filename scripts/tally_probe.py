"""The tally alone on the C2 batch (1M verified votes, 100 signatories): wall
time per hd_tally_device_bitmap call (host syncs included), for the kernel
breakdown run it under rocprofv3 --kernel-trace --stats."""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    import torch
    import hyperdrive_amd as hd
    from hyperdrive_amd import _lib
    from hyperdrive_amd.device import generate, work_stream
    N, S = int(os.environ.get("TP_N", 1 << 20)), int(os.environ.get("TP_S", 100))
    adv = int(os.environ.get("TP_ADV", 0))
    v = hd.Verifier(0)
    sigs, foreign = v.gen_keys(S)
    v.set_signatories(sigs)
    db, _, _ = generate(v, 0, N, S, adv, keys=(sigs, foreign))
    ws = work_stream()
    verdict = torch.empty(N, dtype=torch.uint8, device="cuda")
    bitmap = torch.zeros(N // 32, dtype=torch.int32, device="cuda")
    cb = db.c_struct()
    v.verify_batch_device(cb, verdict.data_ptr(), None, None, bitmap.data_ptr(), ws.cuda_stream)
    ws.synchronize()
    lib = _lib.load()
    t_out, _ = v._tally_struct(N)
    ms = []
    for k in range(int(os.environ.get("TP_CALLS", 20))):
        torch.cuda.synchronize()
        t = time.perf_counter()
        rc = lib.hd_tally_device_bitmap(v.handle, ctypes.byref(cb), bitmap.data_ptr(), ctypes.byref(t_out),
                                        ws.cuda_stream)
        assert rc == 0, rc
        ms.append(round((time.perf_counter() - t) * 1e3, 3))
    print(json.dumps({"n": N, "signers": S, "adv": adv, "tally_ms": ms, "median_ms": sorted(ms)[len(ms) // 2],
                      "n_hr": t_out.n_hr, "n_counts": t_out.n_counts}), flush=True)


if __name__ == "__main__":
    main()
