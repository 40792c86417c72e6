# A/B of table widths: the working-tree library (24-bit G, 20-bit key windows)
# against _lib/var/big (26-bit G, 22-bit key windows, HD_FB_MAX_BYTES raised),
# interleaved, under the kernel trace.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp AB_CALLS=40
for cfg in std big std2 big2; do
  case $cfg in big*) export HD_LIB=hyperdrive_amd/_lib/var/big/libhdverify.so HD_FB_MAX_BYTES=2.3e11 ;; *) unset HD_LIB HD_FB_MAX_BYTES ;; esac
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abb_$cfg -o run -- python3 scripts/ab_fast.py "X=$cfg" > gpurun_out/abb_$cfg.log 2>&1 || exit 1
  grep cfg gpurun_out/abb_$cfg.log | cut -c1-70
  python3 - "$cfg" <<'PY'
import csv,sys,json
rows=list(csv.DictReader(open(f'gpurun_out/abb_{sys.argv[1]}/run_kernel_stats.csv')))
print(' '.join(f"{k}={float(r['AverageNs'])/1e3:.0f}" for r in rows for k in ('k_fast_sums','k_fast_scalars','k_fast_final','k_fast_prep','k_fb_entries') if k in r['Name']))
for l in open(f'gpurun_out/abb_{sys.argv[1]}.log'):
    if l.startswith('{'):
        d=json.loads(l); print('median', d.get('median_last_half_ms'), 'best', d.get('best_ms'), 'hist', d.get('hist'), 'fallback', d.get('fallback_last_call'))
PY
done
