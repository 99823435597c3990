#!/usr/bin/env bash
# The GPU suite in one process (tests -m gpu), then smoke(); logs under gpurun_out/.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 ${LIMIT:-1000} python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread ${SEL:-} > gpurun_out/r4_gpu_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r4_gpu_tests.log; [ $rc = 0 ] || exit 3
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_smoke.log 2>&1 || { tail -5 gpurun_out/r4_smoke.log; exit 3; }
tail -1 gpurun_out/r4_smoke.log
