"""Debug aid (not product code): run scripts/w4_probe_*.so over a golden
fixture and report, per build variant and phase, how many messages differ
between the 3-wave and 4-wave register budgets, and the stage-3 signatories
against the fixture.  Usage: python scripts/w4_probe.py [variant ...]"""
import ctypes
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "..", "tests", "golden", "verify_votes_mix30.npz")


def digests(z):
    out = np.zeros((len(z["type"]), 8), np.uint32)
    for i in range(len(z["type"])):
        h, r = int(z["height"][i]), int(z["round"][i])
        pre = (h & (2**64 - 1)).to_bytes(8, "big") + (r & (2**64 - 1)).to_bytes(8, "big")
        if int(z["type"][i]) == 1:
            pre += (int(z["valid_round"][i]) & (2**64 - 1)).to_bytes(8, "big")
        pre += z["value"][i].tobytes()
        out[i] = np.frombuffer(hashlib.sha256(pre).digest(), ">u4")
    return out


def main():
    z = np.load(GOLDEN)
    keep = np.flatnonzero(np.isin(z["type"], [1, 2, 3]))
    dg = np.ascontiguousarray(digests(z)[keep])
    sig = np.ascontiguousarray(z["sig"][keep])
    frm = np.ascontiguousarray(z["frm"][keep])
    gold_v = z["verdict"][keep]
    gold_rec = z["recovered"][keep]
    n = len(keep)
    variants = sys.argv[1:] or ["base", "nomacc", "nolaunder"]
    report = {}
    for var in variants:
        lib = ctypes.CDLL(os.path.join(HERE, f"w4_probe_{var}.so"))
        lib.probe_run.restype = ctypes.c_int
        lib.probe_run.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint32] + [ctypes.c_void_p] * 5
        lib.probe_host.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_uint32] + [ctypes.c_void_p] * 5
        res = {}
        runs = [(st, 0) for st in (0, 1, 2, 3, 10, 11, 12, 13, 14, 15)]
        runs += [(16, a) for a in (32, 31, 30, 29, 27, 24, 20, 16, 8, 0)] + [(17, a) for a in (32, 30, 27, 24, 0)]
        for stage, arg in runs:
            outs = {}
            for w in (3, 4):
                out = np.zeros((n, 48), np.uint32)
                ver = np.zeros(n, np.uint8)
                rc = lib.probe_run(w, stage, arg, n, dg.ctypes.data, sig.ctypes.data, frm.ctypes.data,
                                   out.ctypes.data, ver.ctypes.data)
                assert rc == 0, rc
                outs[w] = (out, ver)
            out = np.zeros((n, 48), np.uint32)
            ver = np.zeros(n, np.uint8)
            lib.probe_host(stage, arg, n, dg.ctypes.data, sig.ctypes.data, frm.ctypes.data, out.ctypes.data,
                           ver.ctypes.data)
            outs["host"] = (out, ver)
            d = np.flatnonzero((outs[3][0] != outs[4][0]).any(1) | (outs[3][1] != outs[4][1]))
            dh = np.flatnonzero((outs[3][0] != out).any(1) | (outs[3][1] != ver))
            ent = {"differ_3v4": int(len(d)), "differ_3_vs_host": int(len(dh)),
                   "verdicts_w3": np.bincount(outs[3][1], minlength=8).tolist(),
                   "verdicts_host": np.bincount(ver, minlength=8).tolist()}
            if len(dh):
                i = int(dh[0])
                ent["first_vs_host"] = {"i": i, "w3": outs[3][0][i].tolist(), "host": out[i].tolist()}
            if len(d):
                i = int(d[0])
                ent["first"] = {"i": i, "w3": outs[3][0][i].tolist(), "w4": outs[4][0][i].tolist(),
                                "v3": int(outs[3][1][i]), "v4": int(outs[4][1][i])}
            if stage == 3:
                for w in (3, 4, "host"):
                    rec = outs[w][0][:, :8].astype(">u4").view(np.uint8).reshape(n, 32)
                    ok = gold_v == 0
                    ent[f"w{w}_rec_mismatch_on_valid"] = int((rec[ok] != gold_rec[ok]).any(1).sum())
            res[f"{stage}/{arg}"] = ent
            print(var, stage, arg, json.dumps(ent)[:300], flush=True)
        report[var] = res
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/w4_probe.json", "w") as fh:
        json.dump(report, fh, indent=1)


if __name__ == "__main__":
    main()
