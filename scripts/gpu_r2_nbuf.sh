# Bench A/B: pipeline depth (HD_BENCH_NBUF) 3 vs 4 vs 6.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in 3 4 6 3b 4b; do
  export HD_BENCH_NBUF=${cfg%b}
  timeout -k 10 300 python3 bench.py --steps 40 --no-aux --no-sub --no-cpu > gpurun_out/nb_$cfg.json 2> gpurun_out/nb_$cfg.err || { tail -5 gpurun_out/nb_$cfg.err; exit 1; }
  python3 - "$cfg" <<'PY'
import json,sys
for l in open(f'gpurun_out/nb_{sys.argv[1]}.json'):
    if l.startswith('{"metric"'):
        d=json.loads(l); r=d['roofline']
        print(sys.argv[1], round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],3), 'ms/step', 'sums', round(r['kernel_ms'],3), 'call', round(r['verify_call']['ms'],3))
PY
done
