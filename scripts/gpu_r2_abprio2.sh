# Bench A/B: verify / tally stream priorities, interleaved (with the host trace of step starts).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in vh_tn vn_tn vn_th vh_th vh_tn2 vn_th2; do
  case ${cfg%2} in vh_tn) f="--stream-priority high --tally-priority normal" ;; vn_tn) f="--stream-priority normal --tally-priority normal" ;;
                   vn_th) f="--stream-priority normal --tally-priority high" ;; vh_th) f="--stream-priority high --tally-priority high" ;; esac
  timeout -k 10 300 python3 bench.py --steps 40 --no-aux --no-sub --no-cpu $f > gpurun_out/abp2_$cfg.json 2> gpurun_out/abp2_$cfg.err || { tail -5 gpurun_out/abp2_$cfg.err; exit 1; }
  python3 - "$cfg" <<'PY'
import json,sys
for l in open(f'gpurun_out/abp2_{sys.argv[1]}.json'):
    if l.startswith('{"metric"'):
        d=json.loads(l); r=d['roofline']
        print(sys.argv[1], round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],3), 'ms/step', 'sums', round(r['kernel_ms'],3), 'call', round(r['verify_call']['ms'],3))
PY
done
