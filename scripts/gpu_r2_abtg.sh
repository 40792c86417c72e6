# Bench A/B: tally probe-pass grid (HD_TALLY_BPC blocks per CU), interleaved.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in 16 2 4 1 16b 2b; do
  export HD_TALLY_BPC=${cfg%b}
  timeout -k 10 300 python3 bench.py --steps 40 --no-aux --no-sub --no-cpu > gpurun_out/abt_$cfg.json 2> gpurun_out/abt_$cfg.err || { tail -5 gpurun_out/abt_$cfg.err; exit 1; }
  python3 - "$cfg" <<'PY'
import json,sys
for l in open(f'gpurun_out/abt_{sys.argv[1]}.json'):
    if l.startswith('{"metric"'):
        d=json.loads(l); r=d['roofline']
        print(sys.argv[1], round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],3), 'ms/step', 'sums', round(r['kernel_ms'],3), 'call', round(r['verify_call']['ms'],3))
PY
done
