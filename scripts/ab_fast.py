"""A/B of known-key check configurations, one subprocess per configuration.

Each child times hd_verify_batch_device on 1M C2 messages (100 signatories,
optional adversarial share) after a key-learning pass, and reports the best
of several calls plus the verdict histogram.  Usage:
    python scripts/ab_fast.py "HD_FAST_K=0" "HD_FAST_K=16" "HD_FAST_K=8 HD_SUM_WAVES=2" ...
"""
import json
import os
import subprocess
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")


def child():
    sys.path.insert(0, ROOT)
    import torch
    import hyperdrive_amd as hd
    from hyperdrive_amd.device import generate, work_stream
    N, S = int(os.environ.get("AB_N", 1 << 20)), 100
    adv = int(os.environ.get("AB_ADV", 0))
    v = hd.Verifier(0)
    sigs, foreign = v.gen_keys(S)
    v.set_signatories(sigs)
    db, _, _ = generate(v, 0, N, S, adv, keys=(sigs, foreign))
    if os.environ.get("AB_SORT"):
        # messages grouped by signatory (probe of the table reads' locality)
        key = db.frm[:, :8].to(torch.int64)
        k = torch.zeros(N, dtype=torch.int64, device="cuda")
        for b in range(7):
            k = k * 256 + key[:, b]
        perm = torch.argsort(k, stable=True)
        for f in ("type", "height", "round", "valid_round", "value", "frm", "sig"):
            setattr(db, f, getattr(db, f)[perm].contiguous())
    ws = work_stream()
    verdict = torch.empty(N, dtype=torch.uint8, device="cuda")
    cb = db.c_struct()
    ms = []
    hist = None
    for rnd in range(int(os.environ.get("AB_CALLS", 30))):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(ws)
        v.verify_batch_device(cb, verdict.data_ptr(), None, None, None, ws.cuda_stream)
        e1.record(ws)
        e1.synchronize()
        ms.append(round(e0.elapsed_time(e1), 3))
        h = torch.bincount(verdict.to(torch.int64), minlength=8).tolist()
        hist = h if hist is None else hist
        if h != hist:
            hist = "UNSTABLE"
        verdict.fill_(9)
    known, fallback = v.fastpath_stats()
    tail = sorted(ms[len(ms) // 2:])
    print(json.dumps({"cfg": os.environ.get("AB_CFG", ""), "ms": ms[1:], "best_ms": min(ms[1:]),
                      "median_last_half_ms": tail[len(tail) // 2],
                      "known_keys": known, "fallback_last_call": fallback,
                      "msgs_per_s": N / min(ms[1:]) * 1e3, "hist": hist}), flush=True)


if __name__ == "__main__":
    if os.environ.get("AB_CHILD"):
        child()
        sys.exit(0)
    for cfg in sys.argv[1:]:
        env = dict(os.environ, AB_CHILD="1", AB_CFG=cfg)
        for kv in cfg.split():
            k, val = kv.split("=", 1)
            env[k] = val
        r = subprocess.run([sys.executable, __file__], env=env, timeout=300)
        if r.returncode != 0:
            print(json.dumps({"cfg": cfg, "rc": r.returncode}), flush=True)
            sys.exit(r.returncode)
