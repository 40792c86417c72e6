"""Measurement aid (not product code): the tally alone on a verified batch --
hd_tally_device_bitmap called back to back on one stream -- so a
`rocprofv3 --kernel-trace --stats` run shows each tally kernel's own
duration without verify kernels competing for the CUs.

Usage: python scripts/tally_probe.py C2|C3|C5 [calls]"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import hyperdrive_amd as hd
    from hyperdrive_amd import _lib
    from hyperdrive_amd.device import generate, work_stream
    wl = sys.argv[1] if len(sys.argv) > 1 else "C2"
    calls = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    v = hd.Verifier(0)
    ws = work_stream(dev)
    S = 1000 if wl == "C3" else 100
    keys = v.gen_keys(S)
    v.set_signatories(keys[0])
    if wl == "C3":
        n = (64 * (2 * S + 1) + 31) // 32 * 32
        db, _, _ = generate(v, 1, n, S, 0, keys=keys, device=str(dev))
    else:
        n = 1 << 20
        db, _, _ = generate(v, 0, n, S, 30 if wl == "C5" else 0, keys=keys, device=str(dev))
    shard = db.c_struct()
    verdict = torch.empty(n, dtype=torch.uint8, device=dev)
    bitmap = torch.zeros(n // 32, dtype=torch.int32, device=dev)
    for _ in range(2):
        v.verify_batch_device(shard, verdict.data_ptr(), None, None, bitmap.data_ptr(), ws.cuda_stream)
    torch.cuda.synchronize()
    t_out, _ = v._tally_struct(n, pinned=True)
    lib = _lib.load()
    times = []
    for k in range(calls):
        t = time.perf_counter()
        rc = lib.hd_tally_device_bitmap(v.handle, ctypes.byref(shard), bitmap.data_ptr(), ctypes.byref(t_out),
                                        ws.cuda_stream)
        times.append(time.perf_counter() - t)
        assert rc == 0, rc
    times.sort()
    print({"workload": wl, "messages": n, "n_hr": t_out.n_hr, "n_counts": t_out.n_counts,
           "tally_ms_median": round(times[len(times) // 2] * 1e3, 4), "tally_ms_min": round(times[0] * 1e3, 4)},
          flush=True)
    v.close()


if __name__ == "__main__":
    main()
