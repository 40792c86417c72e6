set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp AB_CALLS=40
for cfg in base new; do
  if [ $cfg = base ]; then export HD_LIB=hyperdrive_amd/_lib/var/base/libhdverify.so; else unset HD_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab4_$cfg -o run -- python3 scripts/ab_fast.py "X=$cfg" > gpurun_out/ab4_$cfg.log 2>&1 || exit 1
  grep cfg gpurun_out/ab4_$cfg.log
done
