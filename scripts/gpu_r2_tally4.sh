# The tally alone (base library vs the working tree) under the kernel trace,
# then the default bench step under the kernel trace.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in base new base2 new2; do
  case $cfg in base*) export HD_LIB=hyperdrive_amd/_lib/var/base/libhdverify.so ;; *) unset HD_LIB ;; esac
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tp_$cfg -o run -- \
    python3 scripts/tally_probe.py > gpurun_out/tp_$cfg.log 2>&1 || exit 1
  grep -o '"median_ms[^,]*' gpurun_out/tp_$cfg.log | sed "s/^/$cfg /"
done
unset HD_LIB
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o run -- \
  python3 bench.py --steps 10 --warmup 2 --no-cpu --no-aux --no-sub > gpurun_out/prof_bench.log 2>&1 || exit 2
echo done
