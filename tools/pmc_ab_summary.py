#!/usr/bin/env python3
"""One line per A/B run of PMC passes (tools/measure.sh pmc): bench ms/frame and the dominant kernel's
counters per launch (gpurun_out/pab_<tag>.json, gpurun_out/pmcab_<tag>/*counter_collection.csv).
TD busy = TD_TD_BUSY_sum / (256 TDs x GRBM_GUI_ACTIVE / 8): GRBM_GUI_ACTIVE sums the 8 XCDs' cycles
(9.8 M for a 0.49-ms C4 launch at 2.4 GHz, profiles/traffic_c4.json)."""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    tag = sys.argv[1]
    out = os.path.join(ROOT, "gpurun_out")
    d = json.loads([ln for ln in open(os.path.join(out, f"pab_{tag}.json")) if ln.startswith("{")][-1])
    kern = d["roofline"]["kernel"]
    vals = collections.defaultdict(list)
    for f in glob.glob(os.path.join(out, f"pmcab_{tag}", "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if kern + "<" in row["Kernel_Name"]:
                vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
    avg = {k: sum(v) / len(v) for k, v in vals.items()}
    g = avg.get("GRBM_GUI_ACTIVE", 0.0)
    line = {"tag": tag, "ms_per_frame": d["ms_per_step"], "kernel": kern, "avg_launch_ms": d["roofline"]["avg_launch_ms"],
            "frames_per_launch": d["roofline"]["frames_per_launch"],
            "valu_M": round(avg.get("SQ_INSTS_VALU", 0) / 1e6, 2), "vmem_rd_M": round(avg.get("SQ_INSTS_VMEM_RD", 0) / 1e6, 3),
            "tcp_acc_M": round(avg.get("TCP_TOTAL_CACHE_ACCESSES_sum", 0) / 1e6, 2),
            "waves": int(avg.get("SQ_WAVES", 0)),
            "td_busy": round(avg.get("TD_TD_BUSY_sum", 0) / (g * 32) if g else 0, 3), "launches": len(vals.get("SQ_WAVES", []))}
    print(json.dumps(line), flush=True)
    with open(os.path.join(out, "pmc_ab.jsonl"), "a") as fh:
        fh.write(json.dumps(line) + "\n")


if __name__ == "__main__":
    main()
