export RVGRT_LIB=rvgrt_amd/variants/diag/librvgrt_hip.so
timeout -k 10 200 python tools/flow_waves.py c3 P0 40 > gpurun_out/fw_full.txt 2>&1 || exit 3
opts=$(grep LONGEST_TILE_OPTS gpurun_out/fw_full.txt | awk '{print $2}')
echo "opts $opts"
RV_FLOW_OPTS=$opts timeout -k 10 200 python tools/flow_waves.py c3 P0 40 > gpurun_out/fw_tile.txt 2>&1 || exit 3
RV_FLOW_OPTS=4 timeout -k 10 200 python tools/flow_waves.py c3 P0 40 > gpurun_out/fw_alone.txt 2>&1 || exit 3
