set -o pipefail
export TAG=r06g
timeout -k 10 900 bash tools/measure.sh tests > gpurun_out/r06g_console.txt 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/r06g_smoke.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r06g_driver_bench.log 2>&1
