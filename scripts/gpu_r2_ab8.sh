export TMPDIR=/tmp
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --no-cpu --no-aux > gpurun_out/b_c5i.log 2> gpurun_out/b_c5i.err || { tail -5 gpurun_out/b_c5i.err; exit 1; }
tail -1 gpurun_out/b_c5i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps(d['sub']['C5_ingress_out_of_order'])); print(d['value'], d['ms_per_step'])"
AB_CALLS=30 AB_LIBS="base=hyperdrive_amd/_lib/var/base/libhdverify.so tree=- w2=-@HD_SUM_WAVES=2" bash scripts/gpu_r2_ab7.sh
