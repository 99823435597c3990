cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "in_flight or tiles or cost" > gpurun_out/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/tests.log; [ $rc -le 1 ] || exit 3
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || exit 3
tail -1 gpurun_out/bench.log | cut -c1-400
