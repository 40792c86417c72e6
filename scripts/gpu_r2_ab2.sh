set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 ./scripts/macc_check > gpurun_out/macc.log 2>&1; echo "macc rc=$?" >> gpurun_out/macc.log
cat gpurun_out/macc.log
timeout -k 10 400 python scripts/ab_fast.py "HD_LIB=hyperdrive_amd/_lib/var/base/libhdverify.so" "HD_LIB=hyperdrive_amd/_lib/var/noasm/libhdverify.so" "HD_FAST_K=8" > gpurun_out/ab2.log 2>&1 || exit 2
grep cfg gpurun_out/ab2.log
