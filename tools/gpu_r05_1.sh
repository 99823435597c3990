set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_full_world.py -k "c2 or c4 or 512 or 1024" tests/test_gpu_flow.py > gpurun_out/t1.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/b1.json 2> gpurun_out/b1.err
