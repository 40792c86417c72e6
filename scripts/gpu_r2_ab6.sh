# Fast-path GPU tests on the working tree, then the interleaved verify-call A/B
# of scripts/gpu_r2_ab5.sh (base = _lib/var/base, new = working tree).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_golden.py tests/test_fastpath.py tests/test_gpu_verify.py -m gpu -x -q \
  -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_fast.log 2>&1 || { tail -30 gpurun_out/pytest_fast.log; exit 1; }
tail -2 gpurun_out/pytest_fast.log
SKIP_TESTS=1 bash scripts/gpu_r2_ab5.sh
