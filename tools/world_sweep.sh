set -o pipefail
# C4's frame (3840x2160, reference flags, 2 GI sweeps, UpdateGIData every frame) over cubic world sizes
for w in 8 9 10 11; do
  timeout -k 10 300 python bench.py --config c4 --world $w --steps 100 --warmup 10 --cpu-seconds 0 > gpurun_out/r06wsweep_$w.log 2>&1 || { echo "FAILED $w"; exit 3; }
  grep '^{' gpurun_out/r06wsweep_$w.log | tail -1 >> gpurun_out/r06wsweep.jsonl
  echo "done $w"
done
