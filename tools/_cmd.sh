cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "in_flight or native_loop or tiles" > gpurun_out/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/tests.log; [ $rc -le 1 ] || exit 3
TILES=x STEPS=400 CONFIGS="c2" VARIANTS="main noil main" bash tools/exp_variants.sh 2>&1
HO_K=16 timeout -k 10 300 python tools/host_overhead.py c2 quick > gpurun_out/ho.log 2>&1 || exit 3
grep "native_N8" gpurun_out/ho.log
