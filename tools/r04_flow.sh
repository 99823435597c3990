#!/usr/bin/env bash
# Round 4: flow frames (the drop-in drawCUDA as one k_ref_flow launch) -- parity tests, then bench lines of
# renderLoop's own calls (bench.py --loop drawcuda) with the flow launch and with drawCUDA's two launches.
# Every GPU step under its own time limit; the script stops at the first failure.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
if [ "${TESTS:-1}" = 1 ]; then
  echo "== tests ($(date +%T))"
  timeout -k 10 ${TEST_LIMIT:-400} python -u -m pytest -x -v --timeout 300 --timeout-method thread ${TESTSEL:-tests/test_gpu_flow.py} \
      > gpurun_out/r4_flow_tests.log 2>&1 || { echo "FAILED tests rc=$?"; tail -30 gpurun_out/r4_flow_tests.log; exit 3; }
  tail -3 gpurun_out/r4_flow_tests.log
fi
for c in ${CFGS:-c4 c3 c5}; do
  for flow in ${FLOWS:-1 0}; do
    echo "== $c flow $flow ($(date +%T))"
    timeout -k 10 240 python bench.py --config $c --loop drawcuda --flow $flow --cpu-seconds 0 ${EXTRA:-} \
        > gpurun_out/r4_dc_${c}_f$flow.json 2> gpurun_out/r4_dc_${c}_f$flow.log \
      || { echo "FAILED $c rc=$?"; tail -5 gpurun_out/r4_dc_${c}_f$flow.log; exit 3; }
    python3 -c "import json; d=json.load(open('gpurun_out/r4_dc_${c}_f$flow.json')); print('$c flow $flow', d['ms_per_step'], 'lat', d['latency_ms'], d['kernel_ms']['primary'], d['kernel_ms']['pp_primary'], d['kernel_ms']['gi'], d['roofline']['frac'])"
  done
done
echo "== done"
