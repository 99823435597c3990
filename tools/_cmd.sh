cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for pad in 0 5632 6656 8192 10240; do
RV_LDS_PAD=$pad timeout -k 10 300 python bench.py --cpu-seconds 0 > gpurun_out/pad_$pad.log 2>&1 || exit 3
tail -1 gpurun_out/pad_$pad.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('pad $pad', d['ms_per_step'], d['kernel_ms']['primary'], d['roofline']['frac'])"
done
