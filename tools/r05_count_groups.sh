set -e
mkdir -p gpurun_out/r05h
RT_HEAVY_GROUP=0 RT_LIB_PATH=_variants/librt_count.so timeout -k 10 300 python tools/count_gpu_work.py sphere1m seg > gpurun_out/r05h/count_g0.log 2>&1
RT_HEAVY_GROUP=4 RT_LIB_PATH=_variants/librt_count.so timeout -k 10 300 python tools/count_gpu_work.py sphere1m seg > gpurun_out/r05h/count_g4.log 2>&1
tail -1 gpurun_out/r05h/count_g0.log; tail -1 gpurun_out/r05h/count_g4.log
