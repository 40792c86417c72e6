"""Per-kernel average durations of A/B runs (rocprofv3 --stats CSVs under
gpurun_out/<prefix>*/run_kernel_stats.csv), one column per run."""
import csv
import glob
import os
import sys

pref = sys.argv[1] if len(sys.argv) > 1 else "ab7_"
runs = sorted(glob.glob(os.path.join("gpurun_out", pref + "*", "run_kernel_stats.csv")))
tab, names = {}, []
for p in runs:
    run = os.path.basename(os.path.dirname(p))[len(pref):]
    names.append(run)
    for r in csv.DictReader(open(p)):
        k = r["Name"].split("(")[0].replace("void ", "").replace("(anonymous namespace)::", "")
        if "(anonymous namespace)::" in r["Name"]:
            k = r["Name"].split("(anonymous namespace)::")[1].split("(")[0]
        tab.setdefault(k, {})[run] = float(r["AverageNs"]) / 1e3
print("%-34s" % "kernel (avg us)" + "".join("%10s" % n[:9] for n in names))
for k, row in sorted(tab.items(), key=lambda kv: -max(kv[1].values())):
    if max(row.values()) < 5:
        continue
    print("%-34s" % k[:34] + "".join("%10.1f" % row.get(n, 0.0) for n in names))
