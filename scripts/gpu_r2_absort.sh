# Probe: the verify call on a batch in arrival order vs grouped by signatory
# (locality of the per-key table reads), interleaved, under the kernel trace.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp AB_CALLS=40
for cfg in rnd srt rnd2 srt2; do
  case $cfg in srt*) export AB_SORT=1 ;; *) unset AB_SORT ;; esac
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abs_$cfg -o run -- python3 scripts/ab_fast.py "X=$cfg" > gpurun_out/abs_$cfg.log 2>&1 || exit 1
  python3 - "$cfg" <<'PY'
import csv,sys,json
rows=list(csv.DictReader(open(f'gpurun_out/abs_{sys.argv[1]}/run_kernel_stats.csv')))
print(sys.argv[1], ' '.join(f"{k}={float(r['AverageNs'])/1e3:.0f}" for r in rows for k in ('k_fast_sums','k_fast_scalars','k_fast_final','k_fast_prep') if k in r['Name']))
for l in open(f'gpurun_out/abs_{sys.argv[1]}.log'):
    if l.startswith('{'):
        d=json.loads(l); print('median', d.get('median_last_half_ms'), 'best', d.get('best_ms'), 'hist', d.get('hist'), 'fallback', d.get('fallback_last_call'))
PY
done
