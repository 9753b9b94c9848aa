set -u
RT_LIB_PATH=_variants/librt_count.so timeout -k 10 200 python tools/count_gpu_work.py sphere1m seg > gpurun_out/r02_count44.log 2>&1
