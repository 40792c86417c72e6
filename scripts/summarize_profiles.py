"""Condense rocprofv3 outputs under gpurun_out/ into profiles/<round>/.

profiles/<round>/kernel_stats.csv   rocprofv3 --kernel-trace --stats summary
profiles/<round>/pmc_k_fast_*.json, pmc_known_key_check.json, pmc_k_verify.json
                                    per-launch PMC averages of the known-key check and of
                                    the full recovery, and the
                                    HBM traffic derived per MI355X_MICROARCH.md
                                    (FETCH_SIZE/WRITE_SIZE are KiB; FETCH_SIZE
                                    under-reports wide streaming reads by 2x on
                                    gfx950 -- reported raw and corrected).
"""
import collections
import csv
import json
import os
import shutil
import sys

rnd = sys.argv[1] if len(sys.argv) > 1 else "round1"
src = "gpurun_out"
dst = os.path.join("profiles", rnd)
os.makedirs(dst, exist_ok=True)
shutil.copy(os.path.join(src, "prof", "run_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
def kernel_pmc(match, outname, skip_first=False):
    """per-launch PMC averages of the kernels whose name contains `match`;
    skip_first drops the first dispatch (for k_verify_fast: the warmup call
    that learns the keys, in which every message takes the full recovery)"""
    out = {}
    for name in ("pmc_fetch", "pmc_write", "pmc_stall", "pmc_sq", "pmc_icache"):
        path = os.path.join(src, name, "run_counter_collection.csv")
        if not os.path.exists(path):
            continue
        per = collections.defaultdict(dict)
        meta = {}
        for r in csv.DictReader(open(path)):
            if match not in r["Kernel_Name"]:
                continue
            per[r["Counter_Name"]][int(r["Dispatch_Id"])] = float(r["Counter_Value"])
            meta = {"grid": int(r["Grid_Size"]), "workgroup": int(r["Workgroup_Size"]),
                    "lds": int(r["LDS_Block_Size"]), "scratch": int(r["Scratch_Size"]), "vgpr": int(r["VGPR_Count"]),
                    "sgpr": int(r["SGPR_Count"])}
        for c, byd in per.items():
            vals = [byd[k] for k in sorted(byd)]
            if skip_first and len(vals) > 1:
                vals = vals[1:]
            out[c] = sum(vals) / len(vals)
        if meta:
            out.setdefault("dispatch", meta)
    if not out:
        return
    durs = []
    for r in csv.DictReader(open(os.path.join(src, "prof", "run_kernel_trace.csv"))):
        if match in r["Kernel_Name"]:
            durs.append((int(r["Dispatch_Id"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    durs = [d for _, d in sorted(durs)]
    if skip_first and len(durs) > 1:
        durs = durs[1:]
    if durs:
        out["kernel_stats"] = {"calls": len(durs), "avg_ns": sum(durs) / len(durs), "min_ns": min(durs),
                               "max_ns": max(durs), "first_dispatch_skipped": bool(skip_first)}
    if "FETCH_SIZE" in out and "WRITE_SIZE" in out:
        out["hbm_bytes_raw"] = (out["FETCH_SIZE"] + out["WRITE_SIZE"]) * 1024
        out["hbm_bytes_corrected"] = (2 * out["FETCH_SIZE"] + out["WRITE_SIZE"]) * 1024
    json.dump(out, open(os.path.join(dst, outname), "w"), indent=1)
    print(outname, json.dumps(out, indent=1))
    return out


# the known-key check: its kernels (round 1-2a: prep / scalars / sums / final;
# from round 2b: prep / sinv / sums / zinv / cmp), and their sum per verify call
KK = [k for k in ("k_fast_prep", "k_fast_scalars", "k_fast_sinv", "k_fast_sums", "k_fast_final", "k_fast_zinv",
                  "k_fast_cmp") if any(k in r["Kernel_Name"] for r in csv.DictReader(
                      open(os.path.join(src, "prof", "run_kernel_trace.csv"))))]
parts = [kernel_pmc(k, "pmc_%s.json" % k, skip_first=True) for k in KK]
if all(parts) and all("hbm_bytes_raw" in p for p in parts):
    tot = {"kernels": KK,
           "hbm_bytes_raw": sum(p["hbm_bytes_raw"] for p in parts),
           "hbm_bytes_corrected": sum(p["hbm_bytes_corrected"] for p in parts)}
    if all("kernel_stats" in p for p in parts):
        tot["avg_ns"] = sum(p["kernel_stats"]["avg_ns"] for p in parts)
    for c in ("SQ_WAVE_CYCLES", "SQ_ACTIVE_INST_VALU", "SQ_INSTS_VALU", "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE"):
        if all(c in p for p in parts):
            tot[c] = sum(p[c] for p in parts)
    json.dump(tot, open(os.path.join(dst, "pmc_known_key_check.json"), "w"), indent=1)
    print("pmc_known_key_check.json", json.dumps(tot, indent=1))
kernel_pmc("k_verify<", "pmc_k_verify.json")   # the full recovery (warmup learning pass + empty fallback lists)

# every kernel's per-launch HBM traffic (the aux rows: codec, mq, digest, tally)
allk = collections.defaultdict(lambda: collections.defaultdict(list))
for name in ("pmc_fetch", "pmc_write"):
    path = os.path.join(src, name, "run_counter_collection.csv")
    if not os.path.exists(path):
        continue
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        allk[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
durs = {}
for r in csv.DictReader(open(os.path.join(dst, "kernel_stats.csv"))):
    durs[r["Name"].split("(")[0].replace("void ", "")] = float(r["AverageNs"])
kern = {}
for k, cs in allk.items():
    e = {c: sum(v) / len(v) for c, v in cs.items()}
    e["launches"] = max(len(v) for v in cs.values())
    if "FETCH_SIZE" in e and "WRITE_SIZE" in e:
        e["bytes_raw"] = (e["FETCH_SIZE"] + e["WRITE_SIZE"]) * 1024
        e["bytes_corrected"] = (2 * e["FETCH_SIZE"] + e["WRITE_SIZE"]) * 1024
        if k in durs:
            e["avg_ns"] = durs[k]
            e["GBs_corrected"] = e["bytes_corrected"] / durs[k]
    kern[k] = e
if kern:
    json.dump(kern, open(os.path.join(dst, "pmc_kernels.json"), "w"), indent=1)
