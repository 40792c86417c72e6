# A/B of the split check's messages per lane (HD_FAST_K) on the working-tree
# library, under the kernel trace.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp AB_CALLS=40
for k in 8 16 8 16; do
  export HD_FAST_K=$k
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abk_$k -o run -- python3 scripts/ab_fast.py "K=$k" > gpurun_out/abk_$k.log 2>&1 || exit 1
  grep cfg gpurun_out/abk_$k.log | cut -c1-60
  python3 - "$k" <<'PY'
import csv,sys
rows=list(csv.DictReader(open(f'gpurun_out/abk_{sys.argv[1]}/run_kernel_stats.csv')))
print(' '.join(f"{k}={float(r['AverageNs'])/1e3:.0f}" for r in rows for k in ('k_fast_sums','k_fast_scalars','k_fast_final','k_fast_prep') if k in r['Name']))
PY
done
