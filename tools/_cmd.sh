cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "in_flight or native_loop" > gpurun_out/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/tests.log; [ $rc -le 1 ] || exit 3
for lp in native python; do
timeout -k 10 300 python bench.py --loop $lp > gpurun_out/bench_$lp.log 2>&1 || exit 3
tail -1 gpurun_out/bench_$lp.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lp', d['ms_per_step'], d['fps'], d['value'], d['kernel_ms']['primary'], d['roofline']['frac'])"
done
