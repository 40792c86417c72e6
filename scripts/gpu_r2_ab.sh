set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_fastpath.py tests/test_golden.py tests/test_gpu_verify.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t1.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/t1.log; exit 1; }
tail -3 gpurun_out/t1.log
timeout -k 10 400 python scripts/ab_fast.py "HD_LIB=hyperdrive_amd/_lib/var/base/libhdverify.so" "HD_FAST_K=8" "HD_LIB=hyperdrive_amd/_lib/var/base/libhdverify.so AB_ADV=30" "AB_ADV=30" > gpurun_out/ab1.log 2>&1 || exit 2
cat gpurun_out/ab1.log
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-aux > gpurun_out/bench1.log 2>&1 || exit 3
tail -c 600 gpurun_out/bench1.log
