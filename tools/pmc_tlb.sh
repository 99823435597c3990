#!/usr/bin/env bash
# Address-translation (UTCL1), TD/TCP stall and L1/L2 request counters of one bench loop's dominant kernel
# (three passes, each within the per-block counter limits).  Usage: tools/pmc_tlb.sh CONFIG POSE KERNEL  (on the GPU box)
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
c=$1; pose=${2:-P0}; kern=${3:-k_ref_pipe}
i=0
for set in "TCP_UTCL1_REQUEST_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_SERIALIZATION_STALL_sum TD_COALESCABLE_WAVEFRONT_sum TD_LOAD_WAVEFRONT_sum GRBM_GUI_ACTIVE" \
           "TCP_UTCL1_THRASHING_STALL_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TD_TC_STALL_sum TD_SPI_STALL_sum GRBM_GUI_ACTIVE" \
           "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCP_LATENCY_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"; do
    i=$((i + 1))
    rm -rf "gpurun_out/tlb_${c}_$i"
    timeout -s KILL 150 rocprofv3 --pmc $set --kernel-trace --output-format csv -d "gpurun_out/tlb_${c}_$i" -o run \
        -- python3 bench.py --config "$c" --pose "$pose" --steps 32 --warmup 8 --cpu-seconds 0 --dropin-leg 0 \
        > "gpurun_out/tlb_${c}_$i.log" 2>&1 || { echo "FAILED pass $i"; tail -3 "gpurun_out/tlb_${c}_$i.log"; exit 3; }
done
python3 - "$c" "$kern" <<'PY'
import csv, glob, collections, sys
c, kern = sys.argv[1], sys.argv[2]
vals = collections.defaultdict(list)
for f in glob.glob(f"gpurun_out/tlb_{c}_*/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        if kern in row["Kernel_Name"]:
            vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
for k in sorted(vals):
    v = vals[k]
    print(f"{k:40s} {sum(v) / len(v):16.0f}  ({len(v)} launches)")
PY
