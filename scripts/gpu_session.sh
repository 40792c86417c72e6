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
    probe) run w4_probe 240 python -u scripts/w4_probe.py base ;;
    gtest1) run pytest_gpu1 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "golden or c1 or host_pipeline or routed or multi" ;;
    bench_vs1) HD_BENCH_VSTREAMS=1 run bench_vs1 300 python bench.py --no-cpu --no-aux ;;
    bench_vs2) HD_BENCH_VSTREAMS=2 run bench_vs2 300 python bench.py --no-cpu --no-aux ;;
    bench_vs3) run bench_vs3 300 python bench.py --no-cpu --no-aux ;;
    c5probe) run c5probe 300 python -u scripts/c5_probe.py 5 20 && HD_FOREIGN_KEYS=0 run c5probe_fk0 300 python -u scripts/c5_probe.py 3 20 ;;
    trace_c5) run trace_c5 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_c5 -o run -- python3 scripts/c5_probe.py 2 10 ;;
    bench_thi) run bench_thi 300 python bench.py --no-cpu --no-aux --tally-priority high ;;
    abthi) run bench_thi_a 300 python bench.py --no-cpu --no-aux --tally-priority high && run bench_tlo_a 300 python bench.py --no-cpu --no-aux && run bench_thi_b 300 python bench.py --no-cpu --no-aux --tally-priority high && run bench_tlo_b 300 python bench.py --no-cpu --no-aux ;;
    abk32) AB_VARS="split_k=-1,32;lean_inv=0,1" AB_STREAMS=3 AB_ROUNDS=3 run ab_k32 900 python -u scripts/ab_prio.py C2 C5 C3 ;;
    goldk32) run pytest_goldk32 600 python -u -m pytest tests/test_golden.py tests/test_gpu_verify.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "lean or split_k_32 or adversarial_full" ;;
    c3host) run c3host 300 python -u scripts/c3_host_probe.py 40 && HD_BENCH_VSTREAMS=2 run c3host_vs2 300 python -u scripts/c3_host_probe.py 40 ;;
    abasync) HD_BENCH_ASYNC_TALLY=1 run bench_async_a 300 python bench.py --no-cpu --no-aux && run bench_sync_a 300 python bench.py --no-cpu --no-aux && HD_BENCH_ASYNC_TALLY=1 run bench_async_b 300 python bench.py --no-cpu --no-aux && run bench_sync_b 300 python bench.py --no-cpu --no-aux ;;
    abasync2) run bench_async_thi 300 python bench.py --no-cpu --no-aux --tally-priority high && HD_BENCH_NBUF=8 run bench_async_nb8 300 python bench.py --no-cpu --no-aux && HD_BENCH_NBUF=8 run bench_async_nb8_thi 300 python bench.py --no-cpu --no-aux --tally-priority high ;;
    hosttrace_async) HD_BENCH_ASYNC_TALLY=1 HD_BENCH_HOSTTRACE=1 run hosttrace_async 300 python bench.py --no-cpu --no-aux --no-sub ;;
    abdts) HD_BENCH_ASYNC_TALLY=1 HD_BENCH_DEDICATED_TS=1 run bench_async_dts_a 300 python bench.py --no-cpu --no-aux && HD_BENCH_DEDICATED_TS=1 run bench_thread_dts_a 300 python bench.py --no-cpu --no-aux && run bench_thread_a 300 python bench.py --no-cpu --no-aux && HD_BENCH_ASYNC_TALLY=1 HD_BENCH_DEDICATED_TS=1 run bench_async_dts_b 300 python bench.py --no-cpu --no-aux && HD_BENCH_DEDICATED_TS=1 run bench_thread_dts_b 300 python bench.py --no-cpu --no-aux && run bench_thread_b 300 python bench.py --no-cpu --no-aux ;;
    nullrace) run null_stream_race 300 python -u scripts/null_stream_race.py ;;
    abasync3) HD_BENCH_ASYNC_TALLY=1 HD_BENCH_NBUF=2 run bench_async_nb2 300 python bench.py --no-cpu --no-aux && HD_BENCH_ASYNC_TALLY=1 HD_BENCH_NBUF=3 run bench_async_nb3 300 python bench.py --no-cpu --no-aux && HD_BENCH_ASYNC_TALLY=1 HD_BENCH_NBUF=2 HD_BENCH_HOSTTRACE=1 run hosttrace_async_nb2 300 python bench.py --no-cpu --no-aux --no-sub ;;
    abwarm) run bench_w5a 300 python bench.py --no-cpu --no-aux && run bench_w15 300 python bench.py --no-cpu --no-aux --warmup 15 && run bench_w5b 300 python bench.py --no-cpu --no-aux ;;
    ablean3) AB_VARS="lean_inv=0,1" AB_STREAMS=3 AB_ROUNDS=5 run ab_lean3 900 python -u scripts/ab_prio.py C3 C5 ;;
    abasync4) HD_BENCH_ASYNC_TALLY=2 run bench_async2_a 300 python bench.py --no-cpu --no-aux && run bench_thr_a 300 python bench.py --no-cpu --no-aux && HD_BENCH_ASYNC_TALLY=2 run bench_async2_b 300 python bench.py --no-cpu --no-aux && run bench_thr_b 300 python bench.py --no-cpu --no-aux ;;
    bench_fast) run bench_fast 300 python bench.py --no-cpu --no-aux ;;
    pipe) run pipe_c3 300 python scripts/pipe_probe.py C3 40 && run pipe_c2 300 python scripts/pipe_probe.py C2 30 && run pipe_c5 300 python scripts/pipe_probe.py C5 20 ;;
    tally) run tally_c2 200 python scripts/tally_probe.py C2 && run tally_c3 200 python scripts/tally_probe.py C3 ;;
    tally_trace) run tally_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tally_trace -o run -- python3 scripts/tally_probe.py C2 20 ;;
    trace_c3) run trace_c3 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_c3 -o run -- python3 scripts/pipe_probe.py C3 6 ;;
    rehearse) run rehearse2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --dist-backend gloo --steps 4 --warmup 1 --no-cpu --no-aux --no-sub && run rehearse3_c4 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29562 bench.py --gpus 3 --dist-backend gloo --global-batch 3145728 --steps 3 --warmup 1 --no-cpu --no-aux --no-sub ;;
    trace2) run trace2 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace2 -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu --no-aux --no-sub ;;
    mqtest) run pytest_mq 600 python -u -m pytest tests/test_mq.py tests/test_ingress.py tests/test_c1_network.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    burst) run pytest_burst 300 python -u -m pytest tests/test_gpu_verify.py -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "burst or adversarial" ;;
    golden) run pytest_golden 600 python -u -m pytest tests/test_golden.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    abprio) run ab_prio 900 python -u scripts/ab_prio.py ;;
    absplit) AB_VARS="wave_prio=0,3;split_k=-1,8" AB_STREAMS=2 run ab_split 900 python -u scripts/ab_prio.py ;;
    abtally) AB_VARS="sum_cap=0" AB_STREAMS=1,2 AB_TALLY=on,off,nodup AB_ROUNDS=4 run ab_tally 900 python -u scripts/ab_prio.py C2 C3 ;;
    abcapk) AB_VARS="sum_cap=0,2;split_k=-1,4,8;wave_prio=3" AB_STREAMS=2 run ab_capk 900 python -u scripts/ab_prio.py ;;
    abhwq) AB_VARS="wave_prio=0" AB_STREAMS=1,2 AB_ROUNDS=2 run ab_hwq4 600 python -u scripts/ab_prio.py && GPU_MAX_HW_QUEUES=16 AB_VARS="wave_prio=0" AB_STREAMS=1,2 AB_ROUNDS=2 run ab_hwq16 600 python -u scripts/ab_prio.py && GPU_MAX_HW_QUEUES=16 run ingress_hwq16 300 python -u scripts/ingress_probe.py ;;
    abvprio) AB_VARS="wave_prio=0" AB_STREAMS=1,2 AB_ROUNDS=2 run ab_vprio_hi 600 python -u scripts/ab_prio.py && AB_VPRIO=0 AB_VARS="wave_prio=0" AB_STREAMS=1,2 AB_ROUNDS=2 run ab_vprio_lo 600 python -u scripts/ab_prio.py && AB_VPRIO=0 run ingress_vprio_lo 300 python -u scripts/ingress_probe.py ;;
    tallytest) run pytest_tally 600 python -u -m pytest tests/test_gpu_tally.py tests/test_golden.py tests/test_multi_gpu.py tests/test_ingress.py tests/test_c1_network.py tests/test_mq.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    abtsize) AB_VARS="wave_prio=0" AB_STREAMS=1,2 AB_ROUNDS=3 run ab_tsize_new 600 python -u scripts/ab_prio.py C2 C3 && HD_TALLY_SAFE_TABLES=1 AB_VARS="wave_prio=0" AB_STREAMS=1,2 AB_ROUNDS=3 run ab_tsize_old 600 python -u scripts/ab_prio.py C2 C3 ;;
    ablean) AB_VARS="lean_inv=0,1;sum_cap=0,2" AB_STREAMS=1,2 AB_ROUNDS=3 run ab_lean 900 python -u scripts/ab_prio.py ;;
    trace_lean) HD_LEAN_INV=1 HD_SUM_CAP=2 run trace_lean 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_lean -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu --no-aux --no-sub ;;
    abpairs) AB_VARS="sum_pairs=0,1" AB_STREAMS=1,2 AB_ROUNDS=3 run ab_pairs 900 python -u scripts/ab_prio.py C3 C2 ;;
    abw4) AB_VARS="sum_waves=3,4" AB_STREAMS=1,2 AB_ROUNDS=3 run ab_w4 900 python -u scripts/ab_prio.py ;;
    benchw) run bench_w3a 300 python bench.py --no-cpu --no-aux && HD_SUM_WAVES=4 run bench_w4a 300 python bench.py --no-cpu --no-aux && run bench_w3b 300 python bench.py --no-cpu --no-aux && HD_SUM_WAVES=4 run bench_w4b 300 python bench.py --no-cpu --no-aux ;;
    abcap) AB_VARS="sum_cap=0,2;wave_prio=0,3" AB_STREAMS=1,2 run ab_cap 900 python -u scripts/ab_prio.py ;;
    trace_cap) HD_SUM_CAP=2 HD_WAVE_PRIO=3 run trace_cap 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_cap -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu --no-aux --no-sub ;;
    auth) run pytest_auth 600 python -u -m pytest tests/test_gpu_verify.py tests/test_golden.py tests/test_ingress.py tests/test_c1_network.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "authenticate or ingress or c1" ;;
    foreign) run pytest_foreign 600 python -u -m pytest tests/test_gpu_verify.py tests/test_golden.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "foreign or authenticate or adversarial or burst or matches_golden" ;;
    ingress_fk) HD_FOREIGN_KEYS=16 run ingress_probe_fk 300 python -u scripts/ingress_probe.py ;;
    flushprobe) run flush_probe 300 python -u scripts/flush_probe.py ;;
    ingress) run ingress_probe 300 python -u scripts/ingress_probe.py ;;
    ingress_trace) run ingress_trace 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ingress_trace -o run -- python3 scripts/ingress_probe.py ;;
    pipe2) run pipe_c2 300 python scripts/pipe_probe.py C2 20 ;;
    trace_prio) HD_WAVE_PRIO=3 run trace_prio 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_prio -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu --no-aux --no-sub ;;
    pcie) run pcie 120 scripts/pcie_probe && HSA_ENABLE_SDMA=0 run pcie_nosdma 120 scripts/pcie_probe ;;
    fieldbench) run fieldbench 120 scripts/fieldbench 3 ;;
    fieldbench2) run fieldbench2 120 scripts/fieldbench 2 ;;
    swappc) run swappc 120 scripts/swappc_repro ;;
    gtest_fk) HD_FOREIGN_KEYS=16 run pytest_gpu_fk 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    bench_fk) HD_FOREIGN_KEYS=16 run bench_fk 600 python bench.py ;;
    abxyzz) run ab_xyzz 900 python -u scripts/ab_fast.py "HD_LIB=hyperdrive_amd/_lib/var/libhd_base.so" "HD_SUM_WAVES=3" "HD_SUM_WAVES=2" "HD_LIB=hyperdrive_amd/_lib/var/libhd_base.so" "HD_SUM_WAVES=3" "HD_SUM_WAVES=2" "HD_LIB=hyperdrive_amd/_lib/var/libhd_base.so AB_ADV=30" "HD_SUM_WAVES=3 AB_ADV=30" "HD_SUM_WAVES=2 AB_ADV=30" ;;
    abprof) run ab_prof 900 bash scripts/gpu_ab_prof.sh "base:HD_LIB=hyperdrive_amd/_lib/var/libhd_base.so" "xyzz:HD_SUM_WAVES=0" "base5:HD_LIB=hyperdrive_amd/_lib/var/libhd_base.so AB_ADV=30" "xyzz5:AB_ADV=30" ;;
    abc5) AB_VARS="sum_waves=0,2;verify_waves=3,4" AB_STREAMS=2 AB_ROUNDS=3 run ab_c5 900 python -u scripts/ab_prio.py C5 C2 ;;
    hostpipe) run pytest_host 300 python -u -m pytest tests/test_host_pipeline.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread ;;
    abc5b) AB_VARS="slow_lift=1,0;sum_waves=0,2" AB_STREAMS=2 AB_ROUNDS=3 run ab_c5b 900 python -u scripts/ab_prio.py C5 ;;
    host_trace) run host_trace 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/host_trace -o run -- python3 scripts/host_probe.py ;;
    swappc_bisect) run swappc_nolaunder 120 scripts/swappc_repro_nolaunder ; run swappc_nomacc 120 scripts/swappc_repro_nomacc ; run swappc_noasm 120 scripts/swappc_repro_noasm ;;
    multitest) run pytest_multi 300 python -u -m pytest tests/test_multi_gpu.py tests/test_gpu_tally.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread ;;
    abfused) AB_VARS="fused_cmp=0,1" AB_STREAMS=1,2 AB_ROUNDS=3 run ab_fused 900 python -u scripts/ab_prio.py C2 C5 ;;
    abg26) run ab_g26 900 bash scripts/gpu_ab_prof.sh "g24a:HD_SUM_WAVES=0" "g26a:HD_LIB=hyperdrive_amd/_lib/var/libhd_g26.so" "g24b:HD_SUM_WAVES=0" "g26b:HD_LIB=hyperdrive_amd/_lib/var/libhd_g26.so" ;;
    goldlean) run pytest_goldlean 600 python -u -m pytest tests/test_golden.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "lean" ;;
    abchain) AB_VARS="sum_chain=0,1;sum_cap=0,2;lean_inv=0,1" AB_STREAMS=2,3 AB_ROUNDS=2 run ab_chain 900 python -u scripts/ab_prio.py C2 C5 ;;
    trace_chain) HD_SUM_CHAIN=1 HD_SUM_CAP=2 HD_LEAN_INV=1 run trace_chain 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_chain -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu --no-aux --no-sub ;;
    gtest) run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    gputest) run pytest_gpu 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider ;;
    gputest_all) run pytest_gpu 1200 python -m pytest tests -m gpu -q -p no:cacheprovider ;;
    bench) run bench 600 python bench.py ;;
    smoke) run smoke 300 python __graft_entry__.py smoke ;;
    prof1) HD_BENCH_VSTREAMS=1 run rocprof1 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof1 -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu --no-aux --no-sub ;;
    prof) run rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-aux --no-sub ;;
    pmc_fetch) run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 bench.py --steps 3 --warmup 0 --no-cpu --no-aux --no-sub ;;
    pmc_write) run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python3 bench.py --steps 3 --warmup 0 --no-cpu --no-aux --no-sub ;;
    listc) run list_counters 120 rocprofv3 -L ;;
    pmc_stall) run pmc_stall 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_IFETCH SQ_INSTS_SMEM --output-format csv -d gpurun_out/pmc_stall -o run -- python3 bench.py --steps 3 --warmup 0 --no-cpu --no-aux --no-sub ;;
    pmc_icache) run pmc_icache 600 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_DCACHE_HITS SQC_DCACHE_MISSES --output-format csv -d gpurun_out/pmc_icache -o run -- python3 bench.py --steps 3 --warmup 0 --no-cpu --no-aux --no-sub ;;
    pmc_sq) run pmc_sq 600 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_sq -o run -- python3 bench.py --steps 3 --warmup 0 --no-cpu --no-aux --no-sub ;;
    hiptrace_async) HD_BENCH_ASYNC_TALLY=1 run hiptrace_async 300 rocprofv3 --hip-trace --kernel-trace --output-format csv -d gpurun_out/hiptrace_async -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-aux --no-sub ;;
    routedtest) HD_TALLY_CHECK=1 run pytest_routed 400 python -u -m pytest tests/test_multi_gpu.py tests/test_gpu_tally.py -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread ;;
    tallycheck) HD_TALLY_CHECK=1 run pytest_tallycheck 600 python -u -m pytest tests/test_gpu_tally.py tests/test_golden.py tests/test_multi_gpu.py tests/test_ingress.py tests/test_c1_network.py -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread ;;
    goldsums) run pytest_goldsums 600 python -u -m pytest tests/test_golden.py tests/test_gpu_verify.py tests/test_fastpath.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    absums) run ab_sums 900 bash scripts/gpu_ab_prof.sh "base:HD_LIB=hyperdrive_amd/_lib/var/libhd_r5base.so" "new:HD_SUM_WAVES=0" "base2:HD_LIB=hyperdrive_amd/_lib/var/libhd_r5base.so" "new2:HD_SUM_WAVES=0" "base5:HD_LIB=hyperdrive_amd/_lib/var/libhd_r5base.so AB_ADV=30" "new5:AB_ADV=30" ;;
    absums2) run ab_sums2 900 bash scripts/gpu_ab_prof.sh "base:HD_LIB=hyperdrive_amd/_lib/var/libhd_r5base.so" "p1:HD_LIB=hyperdrive_amd/_lib/var/libhd_r5p1.so" "new:HD_SUM_WAVES=0" "base2:HD_LIB=hyperdrive_amd/_lib/var/libhd_r5base.so" "p1b:HD_LIB=hyperdrive_amd/_lib/var/libhd_r5p1.so" "new2:HD_SUM_WAVES=0" ;;
    absums3) run ab_sums3 900 bash scripts/gpu_ab_prof.sh "p1:HD_LIB=hyperdrive_amd/_lib/var/libhd_r5p1.so" "pp:HD_SUM_WAVES=0" "p1b:HD_LIB=hyperdrive_amd/_lib/var/libhd_r5p1.so" "ppb:HD_SUM_WAVES=0" "pp_pf2:HD_SUM_PF=2" "p1_pf2:HD_LIB=hyperdrive_amd/_lib/var/libhd_r5p1.so HD_SUM_PF=2" ;;
    multinew) HD_TALLY_CHECK=1 run pytest_multinew 400 python -u -m pytest tests/test_multi_gpu.py -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread ;;
    c3async) HD_BENCH_ASYNC_TALLY=1 run c3host_async 300 python -u scripts/c3_host_probe.py 40 ;;
    c3matrix) run c3_sync 300 python -u scripts/c3_host_probe.py 40 && HD_BENCH_NBUF=8 run c3_sync_nb8 300 python -u scripts/c3_host_probe.py 40 && C3_TS_PRIO=-1 run c3_sync_hi 300 python -u scripts/c3_host_probe.py 40 && HD_BENCH_ASYNC_TALLY=1 run c3_async 300 python -u scripts/c3_host_probe.py 40 && HD_BENCH_ASYNC_TALLY=1 C3_TS_PRIO=-1 run c3_async_hi 300 python -u scripts/c3_host_probe.py 40 ;;
    c3trace) run c3trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c3trace -o run -- python3 scripts/c3_host_probe.py 20 ;;
    tally_trace3) run tally_trace3 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tally_trace3 -o run -- python3 scripts/tally_probe.py C3 40 ;;
    c3sync) run c3_sync 300 python -u scripts/c3_host_probe.py 40 ;;
    abhead) HD_LIB=hyperdrive_amd/_lib/var/libhd_r5c.so run bench_old_a 300 python bench.py --no-cpu --no-aux && run bench_new_a 300 python bench.py --no-cpu --no-aux && HD_LIB=hyperdrive_amd/_lib/var/libhd_r5c.so run bench_old_b 300 python bench.py --no-cpu --no-aux && run bench_new_b 300 python bench.py --no-cpu --no-aux ;;
    ing5trace) run ing5trace 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ing5trace -o run -- python3 scripts/ingress_c5_run.py && run ing5 300 python scripts/ingress_c5_run.py ;;
    c3trace_async) HD_BENCH_ASYNC_TALLY=1 run c3trace_async 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/c3trace_async -o run -- python3 scripts/c3_host_probe.py 20 ;;
    evict) run pytest_evict 600 python -u -m pytest tests/test_gpu_verify.py tests/test_golden.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "foreign or evict or authenticate or matches_golden" ;;
    mqpf) run pytest_mqpf 600 python -u -m pytest tests/test_mq.py tests/test_ingress.py tests/test_c1_network.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    mapprobe) run mapped_read_probe 120 scripts/mapped_read_probe ;;
    c3both) run c3_sync 300 python -u scripts/c3_host_probe.py 40 && HD_BENCH_ASYNC_TALLY=1 run c3_async 300 python -u scripts/c3_host_probe.py 40 ;;
    votesprobe) run votes_probe 120 python -u scripts/votes_probe.py ;;
    flushtl) run flush_timeline 300 python -u scripts/flush_timeline.py ;;
    bench_fast2) run bench_fast_a 300 python bench.py --no-cpu --no-aux && run bench_fast_b 300 python bench.py --no-cpu --no-aux ;;
    abchunk) run ing_c0a 300 python scripts/ingress_c5_run.py && HD_INGRESS_CHUNK=262144 run ing_c256a 300 python scripts/ingress_c5_run.py && HD_INGRESS_CHUNK=131072 run ing_c128a 300 python scripts/ingress_c5_run.py && run ing_c0b 300 python scripts/ingress_c5_run.py && HD_INGRESS_CHUNK=262144 run ing_c256b 300 python scripts/ingress_c5_run.py && HD_INGRESS_CHUNK=131072 run ing_c128b 300 python scripts/ingress_c5_run.py ;;
    abcur) run ab_cur 600 bash scripts/gpu_ab_prof.sh "cur:X=1" "cur5:AB_ADV=30" ;;
    abonecall) run ing_two_a 300 python scripts/ingress_c5_run.py && HD_ING_ONECALL=1 run ing_one_a 300 python scripts/ingress_c5_run.py && run bench_two 300 python bench.py --no-cpu --no-aux && HD_ING_ONECALL=1 run bench_one 300 python bench.py --no-cpu --no-aux && run ing_two_b 300 python scripts/ingress_c5_run.py && HD_ING_ONECALL=1 run ing_one_b 300 python scripts/ingress_c5_run.py ;;
    abingorder) run bench_ing_first_a 300 python bench.py --no-cpu --no-aux && HD_BENCH_INGRESS_LAST=1 run bench_ing_last_a 300 python bench.py --no-cpu --no-aux && run bench_ing_first_b 300 python bench.py --no-cpu --no-aux && HD_BENCH_INGRESS_LAST=1 run bench_ing_last_b 300 python bench.py --no-cpu --no-aux ;;
  esac
done
