# The tally alone (scripts/tally_probe.py) under the kernel trace.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tally -o run -- python3 scripts/tally_probe.py > gpurun_out/tally_probe.log 2>&1 || { tail -20 gpurun_out/tally_probe.log; exit 1; }
grep '^{' gpurun_out/tally_probe.log
python3 - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/tally/run_kernel_stats.csv')):
    n = r['Name']
    if any(k in n for k in ('tally', 'rocprim', 'rocclr')):
        print(n[:90], r['Calls'], round(float(r['AverageNs'])/1e3, 1), 'us avg')
PY
