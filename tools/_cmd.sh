cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "trace_bit_exact or frame_parity or gi_ or golden" > gpurun_out/par_main.log 2>&1; rc=$?; echo "parity main rc=$rc"; tail -1 gpurun_out/par_main.log; [ $rc -le 1 ] || exit 3
TILES=x STEPS=200 CONFIGS="c2 c3 c4" VARIANTS="main slp" bash tools/exp_variants.sh 2>&1 | grep -v "tiles_\|frame"
