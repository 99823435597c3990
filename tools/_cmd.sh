cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "in_flight or native_loop or tiles" > gpurun_out/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/tests.log; [ $rc -le 1 ] || exit 3
for cfg in c3 c4; do
timeout -k 10 300 python bench.py --config $cfg --cpu-seconds 0 --steps 50 > gpurun_out/bench_$cfg.log 2>&1 || exit 3
tail -1 gpurun_out/bench_$cfg.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg', d['ms_per_step'], d['fps'], d['value'], d['frames_per_launch'], d['roofline']['frac'])"
done
