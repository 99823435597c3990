#!/usr/bin/env bash
# Round 4: variants of the flow launch (env only), renderLoop's calls (bench.py --loop drawcuda), two runs each:
# name ms/frame k_ref_flow-launch-ms latency flow_fallbacks.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
run() { local name=$1 flow=$2; shift 2
  for rep in 1 2; do
    env "$@" timeout -k 10 200 python bench.py --config ${CFG:-c4} --loop drawcuda --flow $flow --steps 200 --cpu-seconds 0 > gpurun_out/fab_$name.json 2>/dev/null || exit 3
    python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/fab_$name.json') if l.startswith('{')][-1]; print('$name', d['ms_per_step'], d['roofline']['avg_launch_ms'], d['latency_ms'], d.get('flow_fallbacks'))"
  done
}
run base 1 RV_FLOW=1
run own_pp_order 1 RV_FLOW_PP_ORDER=0
run spin0 1 RV_FLOW_SPIN=0
run two_launch 0 RV_FLOW=0
