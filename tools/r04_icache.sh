#!/usr/bin/env bash
# Round 4: instruction-cache behaviour of the C4 launches (pipelined k_ref_pipe, drop-in k_ref_flow): the
# kernels are 62.7 / 72.5 KB of code.  One PMC pass each (4 counters), then tools/pmc_summary.py-style sums.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for loop in native drawcuda; do
  rm -rf gpurun_out/ic_$loop
  timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_WAVES --kernel-trace --output-format csv \
      -d gpurun_out/ic_$loop -o run -- python3 bench.py --loop $loop --steps 32 --warmup 8 --settle 0 --cpu-seconds 0 \
      > gpurun_out/ic_$loop.log 2>&1 || { echo "FAILED $loop"; tail -3 gpurun_out/ic_$loop.log; exit 3; }
  python3 - "$loop" <<'PY'
import csv, glob, sys, collections
loop = sys.argv[1]
f = glob.glob(f"gpurun_out/ic_{loop}/**/run_counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"]
    if "k_ref_pipe" not in k and "k_ref_flow<false" not in k: continue
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    n[(k, r["Counter_Name"])] += 1
for k, d in acc.items():
    launches = max(v for (kk, c), v in n.items() if kk == k)
    h, m = d.get("SQC_ICACHE_HITS", 0), d.get("SQC_ICACHE_MISSES", 0)
    print(loop, k[:60], "launches", launches, {c: round(v / launches) for c, v in d.items()},
          "miss rate", round(m / max(h + m, 1), 4))
PY
done
