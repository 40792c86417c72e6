# GPU tests on the working-tree library, then an interleaved A/B of the verify
# call (base = the library under _lib/var/base, new = the working tree), each
# configuration twice, under the kernel trace.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp AB_CALLS=40
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
  tail -3 gpurun_out/pytest_gpu.log
fi
for cfg in base new base2 new2; do
  case $cfg in base*) export HD_LIB=hyperdrive_amd/_lib/var/base/libhdverify.so ;; *) unset HD_LIB ;; esac
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab5_$cfg -o run -- python3 scripts/ab_fast.py "X=$cfg" > gpurun_out/ab5_$cfg.log 2>&1 || exit 1
  grep cfg gpurun_out/ab5_$cfg.log
done
