set -o pipefail
for r in 1280x720 1920x1080 2560x1440 3840x2160 5120x2880 7680x4320; do
  timeout -k 10 240 python bench.py --config c4 --resolution $r --steps 100 --warmup 10 --cpu-seconds 0 > gpurun_out/r06sweep_$r.log 2>&1 || { echo "FAILED $r"; exit 3; }
  grep '^{' gpurun_out/r06sweep_$r.log | tail -1 >> gpurun_out/r06sweep.jsonl
  echo "done $r"
done
