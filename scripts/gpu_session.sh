#!/bin/bash
# One GPU session: each step under its own time limit; stop at the first step
# that dies abnormally (fault / abort / segfault / timeout), continue past
# plain test failures (exit 1).
mkdir -p gpurun_out
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name" >> gpurun_out/session.log
  timeout -k 10 $secs "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc" >> gpurun_out/session.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "abnormal exit $rc in $name; stopping" >> gpurun_out/session.log; exit $rc; fi
  return 0
}
: > gpurun_out/session.log
for step in "$@"; do
  case $step in
    c5probe) run c5probe 300 python -u scripts/c5_probe.py 5 20 && HD_FOREIGN_KEYS=0 run c5probe_fk0 300 python -u scripts/c5_probe.py 3 20 ;;
    trace_c5) run trace_c5 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_c5 -o run -- python3 scripts/c5_probe.py 2 10 ;;
    nullrace) run null_stream_race 300 python -u scripts/null_stream_race.py ;;
    bench_fast) run bench_fast 300 python bench.py --no-cpu --no-aux ;;
    pipe) run pipe_c3 300 python scripts/pipe_probe.py C3 40 && run pipe_c2 300 python scripts/pipe_probe.py C2 30 && run pipe_c5 300 python scripts/pipe_probe.py C5 20 ;;
    tally) run tally_c2 200 python scripts/tally_probe.py C2 && run tally_c3 200 python scripts/tally_probe.py C3 ;;
    tally_trace) run tally_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tally_trace -o run -- python3 scripts/tally_probe.py C2 20 ;;
    trace_c3) run trace_c3 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_c3 -o run -- python3 scripts/pipe_probe.py C3 6 ;;
    c4adv) run pytest_c4adv 600 python -u -m pytest tests/test_gpu_verify.py -m gpu -x -v -s -p no:cacheprovider --timeout 900 --timeout-method thread -k "c4_16m_adversarial" ;;
    selflaunch) run selflaunch_gloo2 300 python -u bench.py --gpus 2 --dist-backend gloo --steps 4 --warmup 1 --no-cpu --no-aux --no-sub --no-c4-check && (timeout -k 10 120 python bench.py --gpus 2 > gpurun_out/selflaunch_nccl2.log 2>&1; echo "rc=$?" >> gpurun_out/selflaunch_nccl2.log) ;;
    r6tests) run pytest_r6 900 python -u -m pytest tests/test_fastpath.py tests/test_golden.py tests/test_ingress.py tests/test_mq.py tests/test_c1_network.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread && run pytest_r6_zero 300 python -u -m pytest tests/test_gpu_verify.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "zero_window" ;;
    proffull) run proffull 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/proffull -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-aux --no-sub --no-c4-check ;;
    proffinal) run proffinal 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/proffinal -o run -- python3 bench.py --no-cpu --no-aux --no-sub --no-c4-check ;;
    abkw) run ab_kw 900 bash scripts/gpu_ab_prof.sh "kw20a:HD_FB_PW=20" "kw16a:HD_FB_PW=16" "kw13a:HD_FB_PW=13" "kw20b:HD_FB_PW=20" "kw16b:HD_FB_PW=16" "kw13b:HD_FB_PW=13" ;;
    abc3) for rep in a b; do run c3_def_$rep 200 python -u scripts/c3_ab.py def && HD_FAST_K=16 run c3_k16_$rep 200 python -u scripts/c3_ab.py k16 && HD_SUM_WAVES=3 run c3_w3_$rep 200 python -u scripts/c3_ab.py w3 && HD_FAST_K=16 HD_SUM_WAVES=3 run c3_k16w3_$rep 200 python -u scripts/c3_ab.py k16w3 && HD_SUM_WAVES=2 run c3_w2_$rep 200 python -u scripts/c3_ab.py w2; done ;;
    abkw22) run ab_kw22 900 bash scripts/gpu_ab_prof.sh "kw20a:HD_FB_PW=20" "kw22a:HD_LIB=hyperdrive_amd/_lib/var/libhd_kw22.so HD_FB_MAX_BYTES=2.2e11" "kw20b:HD_FB_PW=20" "kw22b:HD_LIB=hyperdrive_amd/_lib/var/libhd_kw22.so HD_FB_MAX_BYTES=2.2e11" ;;
    abg) run ab_g 900 bash scripts/gpu_ab_prof.sh "g24a:HD_SUM_WAVES=0" "g22a:HD_LIB=hyperdrive_amd/_lib/var/libhd_g22.so" "g20a:HD_LIB=hyperdrive_amd/_lib/var/libhd_g20.so" "g24b:HD_SUM_WAVES=0" "g22b:HD_LIB=hyperdrive_amd/_lib/var/libhd_g22.so" "g20b:HD_LIB=hyperdrive_amd/_lib/var/libhd_g20.so" ;;
    distgloo) HD_BENCH_FORCE_DIST=1 HD_BENCH_RANGE_GLOO=1 run distgloo 300 python -u bench.py --no-cpu --no-aux --no-sub --no-c4-check && run nodist 300 python -u bench.py --no-cpu --no-aux --no-sub --no-c4-check && HD_BENCH_FORCE_DIST=1 run distprobe 300 python -u bench.py --no-cpu --no-aux --no-sub --no-c4-check && HD_BENCH_FORCE_DIST=1 HD_BENCH_RANGE_GLOO=1 run distgloo_b 300 python -u bench.py --no-cpu --no-aux --no-sub --no-c4-check ;;
    distprobe) HD_BENCH_FORCE_DIST=1 run distprobe 300 python -u bench.py --no-cpu --no-aux --no-sub --no-c4-check && run nodist 300 python -u bench.py --no-cpu --no-aux --no-sub --no-c4-check && HD_BENCH_FORCE_DIST=1 run distprobe_b 300 python -u bench.py --no-cpu --no-aux --no-sub --no-c4-check && run nodist_b 300 python -u bench.py --no-cpu --no-aux --no-sub --no-c4-check ;;
    rounds) run sums_rounds 300 python -u scripts/sums_rounds_probe.py 20 ;;
    visprobe) run visibility_probe 120 scripts/visibility_probe 20 ;;
    mqpf) run pytest_mqpf 300 python -u -m pytest tests/test_mq.py -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread -k "prefetched" ;;
    rehearse) run rehearse2 300 python bench.py --gpus 2 --dist-backend gloo --steps 4 --warmup 1 --no-cpu --no-aux --no-sub --no-c4-check && run rehearse3_c4 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29562 bench.py --gpus 3 --dist-backend gloo --global-batch 3145728 --steps 3 --warmup 1 --no-cpu --no-aux --no-sub --no-c4-check ;;
    trace2) run trace2 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace2 -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu --no-aux --no-sub --no-c4-check ;;
    mqtest) run pytest_mq 600 python -u -m pytest tests/test_mq.py tests/test_ingress.py tests/test_c1_network.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    burst) run pytest_burst 300 python -u -m pytest tests/test_gpu_verify.py -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "burst or adversarial" ;;
    golden) run pytest_golden 600 python -u -m pytest tests/test_golden.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    auth) run pytest_auth 600 python -u -m pytest tests/test_gpu_verify.py tests/test_golden.py tests/test_ingress.py tests/test_c1_network.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "authenticate or ingress or c1" ;;
    foreign) run pytest_foreign 600 python -u -m pytest tests/test_gpu_verify.py tests/test_golden.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "foreign or authenticate or adversarial or burst or matches_golden" ;;
    flushprobe) run flush_probe 300 python -u scripts/flush_probe.py ;;
    ingress) run ingress_probe 300 python -u scripts/ingress_probe.py ;;
    ingress_trace) run ingress_trace 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ingress_trace -o run -- python3 scripts/ingress_probe.py ;;
    pcie) run pcie 120 scripts/pcie_probe && HSA_ENABLE_SDMA=0 run pcie_nosdma 120 scripts/pcie_probe ;;
    fieldbench) run fieldbench 120 scripts/fieldbench 3 ;;
    hostpipe) run pytest_host 300 python -u -m pytest tests/test_host_pipeline.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread ;;
    host_trace) run host_trace 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/host_trace -o run -- python3 scripts/host_probe.py ;;
    multitest) run pytest_multi 300 python -u -m pytest tests/test_multi_gpu.py tests/test_gpu_tally.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread ;;
    gtest) run pytest_gpu 1120 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    gputest) run pytest_gpu 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider ;;
    gputest_all) run pytest_gpu 1200 python -m pytest tests -m gpu -q -p no:cacheprovider ;;
    bench) run bench 600 python bench.py ;;
    smoke) run smoke 300 python __graft_entry__.py smoke ;;
    prof1) HD_BENCH_VSTREAMS=1 run rocprof1 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof1 -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu --no-aux --no-sub --no-c4-check ;;
    prof) run rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-aux --no-sub --no-c4-check ;;
    pmc_fetch) run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 bench.py --steps 3 --warmup 0 --no-cpu --no-aux --no-sub --no-c4-check ;;
    pmc_write) run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python3 bench.py --steps 3 --warmup 0 --no-cpu --no-aux --no-sub --no-c4-check ;;
    listc) run list_counters 120 rocprofv3 -L ;;
    pmc_stall) run pmc_stall 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_IFETCH SQ_INSTS_SMEM --output-format csv -d gpurun_out/pmc_stall -o run -- python3 bench.py --steps 3 --warmup 0 --no-cpu --no-aux --no-sub --no-c4-check ;;
    pmc_sq) run pmc_sq 600 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_sq -o run -- python3 bench.py --steps 3 --warmup 0 --no-cpu --no-aux --no-sub --no-c4-check ;;
    routedtest) HD_TALLY_CHECK=1 run pytest_routed 400 python -u -m pytest tests/test_multi_gpu.py tests/test_gpu_tally.py -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread ;;
    tallycheck) HD_TALLY_CHECK=1 run pytest_tallycheck 600 python -u -m pytest tests/test_gpu_tally.py tests/test_golden.py tests/test_multi_gpu.py tests/test_ingress.py tests/test_c1_network.py -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread ;;
    goldsums) run pytest_goldsums 600 python -u -m pytest tests/test_golden.py tests/test_gpu_verify.py tests/test_fastpath.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    multinew) HD_TALLY_CHECK=1 run pytest_multinew 400 python -u -m pytest tests/test_multi_gpu.py -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread ;;
    c3trace) run c3trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c3trace -o run -- python3 scripts/c3_host_probe.py 20 ;;
    tally_trace3) run tally_trace3 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tally_trace3 -o run -- python3 scripts/tally_probe.py C3 40 ;;
    c3sync) run c3_sync 300 python -u scripts/c3_host_probe.py 40 ;;
    ing5trace) run ing5trace 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ing5trace -o run -- python3 scripts/ingress_c5_run.py && run ing5 300 python scripts/ingress_c5_run.py ;;
    evict) run pytest_evict 600 python -u -m pytest tests/test_gpu_verify.py tests/test_golden.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "foreign or evict or authenticate or matches_golden" ;;
  esac
done
