cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for k in 8 16; do
timeout -k 10 300 python bench.py --inflight $k --cpu-seconds 0 > gpurun_out/b_$k.log 2>&1 || exit 3
tail -1 gpurun_out/b_$k.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('streams 1 inflight $k', d['ms_per_step'], d['fps'], d['value'], d['kernel_ms']['primary'], d['roofline']['frac'])"
done
HO_K=8,16,32 timeout -k 10 300 python tools/host_overhead.py c2 quick > gpurun_out/ho.log 2>&1 || exit 3
grep "native_N8\|native_N1" gpurun_out/ho.log
