"""Measurement aid (not product code): one bench workload through bench.py's
Pipeline, N verify streams and the threaded tally vs variants, printing
ms/step per setting -- run it under `rocprofv3 --kernel-trace` to see how
consecutive verify calls overlap.

Usage: python scripts/pipe_probe.py C2|C3|C5 [steps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    import hyperdrive_amd as hd
    from hyperdrive_amd.device import generate, work_stream
    wl = sys.argv[1] if len(sys.argv) > 1 else "C3"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    v = hd.Verifier(0)
    ws_hi = work_stream(dev, priority=-1)
    ws_lo = torch.cuda.Stream(device=dev, priority=0)
    ts_hi = torch.cuda.Stream(device=dev, priority=-1)
    ts_lo = torch.cuda.Stream(device=dev, priority=0)
    S = 1000 if wl == "C3" else 100
    keys = v.gen_keys(S)
    v.set_signatories(keys[0])
    if wl == "C3":
        n = (64 * (2 * S + 1) + 31) // 32 * 32
        db, _, _ = generate(v, 1, n, S, 0, keys=keys, device=str(dev))
    else:
        n = 1 << 20
        db, _, _ = generate(v, 0, n, S, 30 if wl == "C5" else 0, keys=keys, device=str(dev))
    res = {}
    # (verify streams, tally on, verify priority high, tally priority high)
    settings = [(1, False, True, False), (1, True, True, False), (1, True, False, True),
                (2, False, True, False), (2, True, True, False), (2, True, False, True),
                (3, False, True, False), (3, True, True, False), (3, True, False, True)]
    for vs, tally, vhi, thi in settings:
        bench.Pipeline.VSTREAMS = vs
        p = bench.Pipeline(v, db, n, 0, 0, 1, None, ws_hi if vhi else ws_lo, ts_hi if thi else ts_lo, tally=tally)
        p.run(3)
        el = bench.timed(p, steps, None, dev)
        key = f"vs{vs}_" + (("tally_" + ("thi" if thi else "vhi")) if tally else "notally")
        res[key] = round(el / steps * 1e3, 4)
        print(wl, key, res[key], flush=True)
    print({"workload": wl, "messages": n, "ms_per_step": res}, flush=True)
    v.close()


if __name__ == "__main__":
    main()
