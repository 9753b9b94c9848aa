set -u
RT_LIB_PATH=_variants/librt_tt.so timeout -k 10 200 python tools/tile_times.py > gpurun_out/r02_tiles9.log 2>&1
