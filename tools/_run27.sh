set -u
RT_DEBUG_WAVES=1 RT_LIB_PATH=_variants/librt_ws.so timeout -k 10 200 python tools/wave_stats.py > gpurun_out/r02_waves27.log 2>&1
RT_LIB_PATH=_variants/librt_count.so timeout -k 10 200 python tools/count_gpu_work.py sphere1m > gpurun_out/r02_count27.log 2>&1
