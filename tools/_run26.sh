set -u
RT_DEBUG_WAVES=1 RT_LIB_PATH=_variants/librt_ws.so timeout -k 10 200 python tools/wave_stats.py > gpurun_out/r02_waves26.log 2>&1
