# Interleaved verify-call A/B of several libraries under the kernel trace:
# AB_LIBS="name=path[@VAR=val,VAR=val] ..." (path "-" = the working tree's
# library; the optional environment goes to that configuration only), each run
# twice in turn.  Fast-path GPU tests on the working tree first unless SKIP_TESTS=1.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp AB_CALLS=${AB_CALLS:-40}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests/test_golden.py tests/test_fastpath.py tests/test_gpu_verify.py -m gpu -x -q \
    -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_fast.log 2>&1 || { tail -30 gpurun_out/pytest_fast.log; exit 1; }
  tail -2 gpurun_out/pytest_fast.log
fi
for rep in 1 2; do
  for spec in $AB_LIBS; do
    name=${spec%%=*}; rest=${spec#*=}; path=${rest%%@*}; envs=""
    [ "$rest" != "$path" ] && envs=$(echo "${rest#*@}" | tr ',' ' ')
    if [ "$path" = "-" ]; then unset HD_LIB; else export HD_LIB=$path; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab7_${name}_$rep -o run -- \
      python3 scripts/ab_fast.py "X=${name}_$rep $envs" > gpurun_out/ab7_${name}_$rep.log 2>&1 || exit 1
    grep cfg gpurun_out/ab7_${name}_$rep.log | cut -c1-60
    grep -o '"best_ms[^,]*, "median_last_half_ms[^,]*' gpurun_out/ab7_${name}_$rep.log
  done
done
