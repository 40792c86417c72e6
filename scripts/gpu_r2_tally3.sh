# Tally/multi GPU tests, the tally probe, the N>1 rehearsal and the dup A/B.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_tally.py tests/test_golden.py tests/test_multi_gpu.py tests/test_ingress.py tests/test_gpu_verify.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_tally.log 2>&1 || { tail -40 gpurun_out/pytest_tally.log; exit 1; }
tail -2 gpurun_out/pytest_tally.log
bash scripts/gpu_r2_tally.sh && bash scripts/gpu_r2_rehearse.sh && bash scripts/gpu_r2_abdup.sh
