set -u
RT_LIB_PATH=_variants/librt_pc.so timeout -k 10 200 python tools/pixel_work.py 210,294 174,155 59,294 > gpurun_out/r02_pixwork11.log 2>&1
RT_LIB_PATH=_variants/librt_tt.so timeout -k 10 200 python tools/tile_times.py > gpurun_out/r02_tiles11.log 2>&1
