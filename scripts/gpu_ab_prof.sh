#!/bin/bash
# A/B of verify-call variants: each "name:ENV=VAL ENV=VAL" runs scripts/ab_fast.py
# under rocprofv3 --kernel-trace --stats; per-kernel averages land in
# gpurun_out/ab_<name>/ and the call timings in gpurun_out/ab_<name>.log
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp AB_CALLS=${AB_CALLS:-40}
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  env $envs timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab_$name -o run -- python3 scripts/ab_fast.py "X=$name" > gpurun_out/ab_$name.log 2>&1 || { tail -5 gpurun_out/ab_$name.log; exit 1; }
  grep '"cfg"' gpurun_out/ab_$name.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', 'best', d['best_ms'], 'median', d['median_last_half_ms'], 'fallback', d['fallback_last_call'], d['hist'][:2])"
  python3 - <<PY
import csv, glob
f = glob.glob('gpurun_out/ab_$name/**/*kernel_stats.csv', recursive=True)[0]
for x in csv.DictReader(open(f)):
    if 'fast' in x['Name'] or 'k_verify<' in x['Name']:
        print('   ', x['Name'].split('(')[0][-40:], x['Calls'], round(float(x['AverageNs'])/1e3, 1), 'us')
PY
done
