set -u
RT_LIB_PATH=_variants/librt_pc.so timeout -k 10 200 python tools/pixel_work.py > gpurun_out/r02_pixwork10.log 2>&1
