"""bench.py's C3 line on its own (1,000 signatories, 64 rounds of 1 propose +
1,000 prevotes + 1,000 precommits = 128,064 messages; 3 verify streams and
the tally thread, 160 timed steps) for A/B of context variants set through
the environment (HD_FAST_K, HD_SUM_WAVES, ...: include/hd_verify.h).  One
JSON line.  Usage: HD_FAST_K=16 python scripts/c3_ab.py [label]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    import hyperdrive_amd as hd
    from hyperdrive_amd.device import generate, work_stream
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    ws = work_stream(dev, priority=-1)
    torch.cuda.set_stream(ws)
    ts = torch.cuda.Stream(device=dev, priority=0)
    v = hd.Verifier(0)
    S = 1000
    k3 = v.gen_keys(S)
    v.set_signatories(k3[0])
    n = (64 * (2 * S + 1) + 31) // 32 * 32
    db, _, _ = generate(v, 1, n, S, 0, keys=k3, device=str(dev))
    p = bench.Pipeline(v, db, n, 0, 0, 1, None, ws, ts)
    p.run(1)
    torch.cuda.synchronize(dev)
    p.run(8)
    steps = 160
    rates = []
    for _ in range(3):
        el = bench.timed(p, steps, None, dev)
        rates.append(n * steps / el)
    vd, _, _ = p.last(steps)
    print(json.dumps({"label": sys.argv[1] if len(sys.argv) > 1 else "", "msgs_per_s": sorted(rates)[1],
                      "all": [round(r / 1e6, 1) for r in rates], "valid": int((vd == 0).sum()), "messages": n,
                      "geometry": v.fastpath_geometry(), "fallback": v.fastpath_stats()[1],
                      "env": {k: os.environ[k] for k in os.environ if k.startswith("HD_")}}), flush=True)
    p.close()
    v.close()


if __name__ == "__main__":
    main()
