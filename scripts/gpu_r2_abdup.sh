# Bench A/B: tally with and without the per-message dup download.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in dup nodup dup2 nodup2 notally; do
  unset HD_BENCH_NO_DUP; f=""
  case $cfg in nodup*) export HD_BENCH_NO_DUP=1 ;; notally) f="--no-tally" ;; esac
  timeout -k 10 300 python3 bench.py --steps 40 --no-aux --no-sub --no-cpu $f > gpurun_out/abd_$cfg.json 2> gpurun_out/abd_$cfg.err || { tail -5 gpurun_out/abd_$cfg.err; exit 1; }
  python3 - "$cfg" <<'PY'
import json,sys
for l in open(f'gpurun_out/abd_{sys.argv[1]}.json'):
    if l.startswith('{"metric"'):
        d=json.loads(l); r=d['roofline']
        print(sys.argv[1], round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],3), 'ms/step', 'sums', round(r['kernel_ms'],3), 'call', round(r['verify_call']['ms'],3))
PY
done
