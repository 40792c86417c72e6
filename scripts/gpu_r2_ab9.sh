# Full-recovery GPU parity (verify / golden / fast path / tally), then the
# 30 % adversarial verify call with the recovery's u1 G from the fixed-base G
# table (default) vs the GLV ladder's own G table (HD_RECOVER_GLV_G=1).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_verify.py tests/test_golden.py tests/test_fastpath.py tests/test_gpu_tally.py -m gpu -x -q \
  -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_rec.log 2>&1 || { tail -30 gpurun_out/pytest_rec.log; exit 1; }
tail -2 gpurun_out/pytest_rec.log
AB_ADV=30 SKIP_TESTS=1 AB_CALLS=20 AB_LIBS="fbg=- glv=-@HD_RECOVER_GLV_G=1" bash scripts/gpu_r2_ab7.sh
