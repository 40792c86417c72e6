"""Where a verify step's time goes between consecutive k_fast_sums launches,
from a rocprofv3 --kernel-trace CSV (e.g. gpurun_out/trace2/run_kernel_trace.csv
of `bench.py` on two verify streams): per gap, its length and the kernels
that ran (or started) in it; and the share of the timeline with a k_fast_sums
running.  Usage: python scripts/trace_gaps.py <run_kernel_trace.csv> [last_n_gaps]"""
import csv
import sys


def name(k):
    k = k.replace("(anonymous namespace)::", "").replace("void ", "")
    return k.split("(")[0]


rows = list(csv.DictReader(open(sys.argv[1])))
last = int(sys.argv[2]) if len(sys.argv) > 2 else 8
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name(r["Kernel_Name"]), r["Stream_Id"]) for r in rows)
sums = [e for e in ev if e[2].startswith("k_fast_sums")]
if len(sums) < 3:
    sys.exit("fewer than 3 k_fast_sums launches")
t0, t1 = sums[-last - 1][0], sums[-1][1]
busy, cur = 0, None
for s, e, _, _ in sorted((e for e in sums if e[0] >= t0), key=lambda x: x[0]):
    if cur is None or s > cur[1]:
        if cur:
            busy += cur[1] - cur[0]
        cur = [s, e]
    else:
        cur[1] = max(cur[1], e)
busy += cur[1] - cur[0]
print(f"window {(t1 - t0) / 1e3:.1f} us, k_fast_sums running {busy / (t1 - t0):.3f} of it")
for a, b in zip(sums[-last - 1:-1], sums[-last:]):
    gap = (b[0] - a[1]) / 1e3
    inside = [f"{e[2][:16]}@s{e[3]}:{(e[1] - e[0]) / 1e3:.0f}" for e in ev if a[1] <= e[0] < b[0]]
    print(f"sums s{a[3]} {(a[1] - a[0]) / 1e3:7.1f} us | gap {gap:7.1f} us | " + " ".join(inside))
