#!/usr/bin/env bash
# Round-3 A/B runs on the GPU box: bench lines per variant, one log each under gpurun_out/ab_<tag>.log.
# usage: bash tools/r03_ab.sh "<tag>|<bench args>" ...   (each run under its own time limit; stops at the
# first failure)
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for spec in "$@"; do
    tag=${spec%%|*}; args=${spec#*|}
    echo "== $tag: $args ($(date +%T))"
    timeout -k 10 ${AB_LIMIT:-240} python bench.py --cpu-seconds 0 $args > gpurun_out/ab_$tag.log 2>&1 \
        || { rc=$?; echo "FAILED $tag rc=$rc"; tail -5 gpurun_out/ab_$tag.log; exit 3; }
    python - gpurun_out/ab_$tag.log <<'PY'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
d = json.loads(line); ro = d["roofline"]
print(f"   ms/frame {d['ms_per_step']:.4f}  Mrays/s {d['value']:.0f}  kernel {ro['kernel']} {ro['avg_launch_ms']:.4f} ms"
      f" x{ro['frames_per_launch']}  frac {ro['frac']:.4f}  stage_ms {d['stage_ms']}")
PY
done
