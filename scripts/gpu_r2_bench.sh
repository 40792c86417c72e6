#!/bin/bash
# round-2 GPU session: partition/tally tests, the default bench line, a kernel trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_multi_gpu.py tests/test_gpu_tally.py tests/test_gpu_verify.py tests/test_golden.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t4.log 2>&1 || { tail -30 gpurun_out/t4.log; exit 1; }
tail -2 gpurun_out/t4.log
timeout -k 10 600 python bench.py > gpurun_out/bench_r2.json 2> gpurun_out/bench_r2.err || { tail -20 gpurun_out/bench_r2.err; exit 2; }
cat gpurun_out/bench_r2.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r2 -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu --no-aux --no-sub > gpurun_out/prof_r2.log 2>&1 || { tail -20 gpurun_out/prof_r2.log; exit 3; }
echo done
