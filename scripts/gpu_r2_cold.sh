# GPU tests (-x) and the cold-start probe on the working-tree library.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cold -o run -- python3 scripts/cold_probe.py > gpurun_out/cold_probe.log 2>&1 || { tail -20 gpurun_out/cold_probe.log; exit 1; }
grep '^{' gpurun_out/cold_probe.log
python3 - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/cold/run_kernel_stats.csv')):
    if any(k in r['Name'] for k in ('k_fb_', 'k_verify<', 'k_fast_sums')):
        print(r['Name'][:60], r['Calls'], round(float(r['TotalDurationNs'])/1e6, 2), 'ms total', round(float(r['MaxNs'])/1e6, 2), 'ms max')
PY
