#!/usr/bin/env bash
# Per library variant (VARIANTS="main gint ..."; main = rvgrt_amd/librvgrt_hip.so, others
# rvgrt_amd/variants/<v>/): a bench line (STEPS frames of CONFIG) and one rocprofv3 PMC pass of
# COUNTERS over a short run, averaged per k_ref_pipe launch.  One GPU step per command, each under
# its own time limit; stops at the first failure.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cfg=${CONFIG:-c4}
for v in ${VARIANTS:-main}; do
  lib=""; [ "$v" != main ] && lib=$PWD/rvgrt_amd/variants/$v/librvgrt_hip.so
  out=gpurun_out/pv_${v}_${cfg}
  RVGRT_LIB=$lib timeout -k 10 300 python bench.py --config $cfg --steps ${STEPS:-100} --warmup 5 --cpu-seconds 0 \
      > $out.json 2> $out.err || exit 3
  rm -rf gpurun_out/pmcv_$v
  RVGRT_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc ${COUNTERS:-FETCH_SIZE} --kernel-trace --output-format csv \
      -d gpurun_out/pmcv_$v -o run -- python3 bench.py --config $cfg --steps 16 --warmup 8 --cpu-seconds 0 \
      > $out.pmc.log 2>&1 || exit 3
  python3 - "$v" "$out.json" gpurun_out/pmcv_$v <<'PY'
import csv, glob, json, sys, collections
v, js, d = sys.argv[1:4]
b = json.load(open(js))
rows = []
for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        if "k_ref_pipe" in row["Kernel_Name"] or "k_render" in row["Kernel_Name"]:
            rows.append(row)
# the launches of the largest grid (full frame groups / whole pipelined frames)
gmax = max(int(r.get("Grid_Size", 0)) for r in rows)
vals = collections.defaultdict(list)
for r in rows:
    if int(r.get("Grid_Size", 0)) == gmax:
        vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
avg = {k: round(sum(x) / len(x) / 1024.0 * (2 if k == "FETCH_SIZE" else 1), 1) for k, x in vals.items() if x}
fpl = b["frames_per_launch"].get("primary", 1)
print(v, "ms", b["ms_per_step"], "kernel", b["kernel_ms"]["primary"], "frames/launch", fpl, "grid", gmax,
      "MiB/launch", avg, "MiB/frame", {k: round(x / fpl, 2) for k, x in avg.items()})
PY
done
