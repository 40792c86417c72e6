"""Fold rocprofv3 --pmc passes (separate runs: FETCH_SIZE, WRITE_SIZE, an SQ
set) of `bench.py --steps 3 --warmup 0 --no-cpu --no-aux --no-sub` into the
per-launch JSON that bench.py's pmc_traffic() reads:

    python scripts/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/pmc_sq profiles/round5

k_fast_sums (the 1M-message launches: the grid of the headline batch) and the
known-key check (every kernel of one verify call: k_fast_prep, k_fast_sinv,
k_fast_sums, k_fast_zinv, k_fast_cmp, k_slow_lift, k_verify) averaged per
launch / per call.  FETCH_SIZE and WRITE_SIZE are KiB; on gfx950 FETCH_SIZE
reports half the bytes of a wide coalesced read (MI355X_MICROARCH.md), so
hbm_bytes_corrected = 2 FETCH + WRITE.  The first dispatch of each kernel is
skipped (table builds and cold caches)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

CHECK = ("k_fast_prep", "k_fast_sinv", "k_fast_sums", "k_fast_zinv", "k_fast_cmp", "k_slow_lift", "k_verify<")


def load(d):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    rows = defaultdict(dict)   # dispatch -> {counter: value, name, grid, ...}
    for r in csv.DictReader(open(f)):
        e = rows[int(r["Dispatch_Id"])]
        e["name"] = r["Kernel_Name"]
        e["grid"] = int(r["Grid_Size"])
        e["meta"] = {"grid": int(r["Grid_Size"]), "workgroup": int(r["Workgroup_Size"]),
                     "lds": int(r["LDS_Block_Size"]), "scratch": int(r["Scratch_Size"]),
                     "vgpr": int(r["VGPR_Count"]), "sgpr": int(r["SGPR_Count"])}
        e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        e["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return rows


def main():
    fetch, write, sq, out = sys.argv[1:5]
    passes = [load(d) for d in (fetch, write, sq)]
    sums = defaultdict(list)
    check = defaultdict(float)
    ncalls = 0
    meta = None
    for rows in passes:
        seen = set()
        for did in sorted(rows):
            e = rows[did]
            if "k_fast_sums" in e["name"] and e["grid"] >= (1 << 20) // 4:
                if "k_fast_sums" not in seen:
                    seen.add("k_fast_sums")
                    continue
                meta = e["meta"]
                for k, v in e.items():
                    if k.isupper():
                        sums[k].append(v)
                sums["ns"].append(e["ns"])
    res = {k: sum(v) / len(v) for k, v in sums.items() if k != "ns"}
    res["dispatch"] = meta
    res["kernel_stats"] = {"calls": len(sums["ns"]), "avg_ns": sum(sums["ns"]) / max(1, len(sums["ns"])),
                           "first_dispatch_skipped": True}
    res["hbm_bytes_raw"] = (res["FETCH_SIZE"] + res["WRITE_SIZE"]) * 1024
    res["hbm_bytes_corrected"] = (2 * res["FETCH_SIZE"] + res["WRITE_SIZE"]) * 1024
    # the whole check per call: every check kernel's bytes, divided by the sums launches
    for counter, rows in (("FETCH_SIZE", passes[0]), ("WRITE_SIZE", passes[1])):
        skipped = set()
        tot, calls = 0.0, 0
        for did in sorted(rows):
            e = rows[did]
            kn = next((k for k in CHECK if k in e["name"]), None)
            if kn is None:
                continue
            if kn not in skipped:
                skipped.add(kn)
                continue
            tot += e.get(counter, 0.0)
            calls += kn == "k_fast_sums"
        check[counter] = tot / max(1, calls)
        ncalls = calls
    call = {"FETCH_SIZE": check["FETCH_SIZE"], "WRITE_SIZE": check["WRITE_SIZE"], "calls": ncalls,
            "kernels": list(CHECK),
            "hbm_bytes_raw": (check["FETCH_SIZE"] + check["WRITE_SIZE"]) * 1024,
            "hbm_bytes_corrected": (2 * check["FETCH_SIZE"] + check["WRITE_SIZE"]) * 1024}
    os.makedirs(out, exist_ok=True)
    json.dump(res, open(os.path.join(out, "pmc_k_fast_sums.json"), "w"), indent=1)
    json.dump(call, open(os.path.join(out, "pmc_known_key_check.json"), "w"), indent=1)
    print(json.dumps({"sums": {k: res[k] for k in ("hbm_bytes_raw", "hbm_bytes_corrected")},
                      "check": {k: call[k] for k in ("hbm_bytes_raw", "hbm_bytes_corrected", "calls")}}))


if __name__ == "__main__":
    main()
