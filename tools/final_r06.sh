set -o pipefail
export TAG=r06f
timeout -k 10 600 bash tools/measure.sh tests > gpurun_out/r06f_console.txt 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/r06f_smoke.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r06f_driver_bench.log 2>&1 &&
timeout -k 10 900 bash tools/measure.sh bench c1:--config_c1 c2:--config_c2 c3:--config_c3 c4:--config_c4 c5:--config_c5 c3_P1:--config_c3_--pose_P1 c4_P1:--config_c4_--pose_P1 c5_P1:--config_c5_--pose_P1 >> gpurun_out/r06f_console.txt 2>&1 &&
timeout -k 10 400 bash tools/measure.sh prof >> gpurun_out/r06f_console.txt 2>&1
