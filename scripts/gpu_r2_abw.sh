# A/B of k_fast_sums occupancy (HD_SUM_WAVES 3 vs 2), interleaved, kernel trace.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp AB_CALLS=40
for w in 3 2 3b 2b; do
  export HD_SUM_WAVES=${w%b}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abw_$w -o run -- python3 scripts/ab_fast.py "W=$w" > gpurun_out/abw_$w.log 2>&1 || exit 1
  python3 - "$w" <<'PY'
import csv,sys,json
rows=list(csv.DictReader(open(f'gpurun_out/abw_{sys.argv[1]}/run_kernel_stats.csv')))
print(sys.argv[1], ' '.join(f"{k}={float(r['AverageNs'])/1e3:.0f}" for r in rows for k in ('k_fast_sums','k_fast_scalars','k_fast_final','k_fast_prep') if k in r['Name']))
for l in open(f'gpurun_out/abw_{sys.argv[1]}.log'):
    if l.startswith('{'):
        d=json.loads(l); print('median', d.get('median_last_half_ms'), 'best', d.get('best_ms'), 'hist', d.get('hist'))
PY
done
