#!/usr/bin/env bash
# Round 4: C3 grouped launch (k_ref_group, 8 frames per launch) memory-side traffic with the GI bounce hits'
# texture tile from the table (main) and from the noise (rvgrt_amd/variants/gitexnoise), FETCH/WRITE passes.
cd "$(dirname "$0")/.." || exit 1
for v in main gitexnoise; do lib=""; [ "$v" != main ] && lib=$PWD/rvgrt_amd/variants/$v/librvgrt_hip.so
  for set in FETCH_SIZE WRITE_SIZE; do
    rm -rf gpurun_out/pmc_gx${v}_$set
    RVGRT_LIB=$lib timeout -s KILL 150 rocprofv3 --pmc $set --kernel-trace --output-format csv -d gpurun_out/pmc_gx${v}_$set -o run -- \
        python3 bench.py --config c3 --steps 32 --warmup 8 --cpu-seconds 0 > gpurun_out/gx_pmc_${v}_$set.log 2>&1 || exit 3
  done
  python3 tools/pmc_summary.py --prefix gx${v}_ --config c3 --kernel k_ref_group --fpl 8 --grid -1 --out gpurun_out/traffic_c3_gx_$v.json || exit 3
done
for rep in 1 2; do for v in main gitexnoise; do lib=""; [ "$v" != main ] && lib=$PWD/rvgrt_amd/variants/$v/librvgrt_hip.so
  RVGRT_LIB=$lib timeout -k 10 200 python bench.py --config c3 --steps 400 --cpu-seconds 0 > gpurun_out/gx_$v.json 2>/dev/null || exit 3
  python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/gx_$v.json') if l.startswith('{')][-1]; print('c3 $v', d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['algorithmic_bytes_per_launch'])"
done; done
